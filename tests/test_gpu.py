"""GPU parity tests (MI355X) of the production paths: every golden vector of the compiled reference through
the C ABI under the library's default policy, plus multi-stripe round trips checked against the CPU oracle.
The non-default kernel variants (options of the release library, and the A/B families of the diagnostic
library) run the same checks afterwards, in tests/test_gpu_variants.py, so that no option-only family can
hide the production path behind a failure.

All tests run in one process; they need librs_amd.so built for gfx950 (no CPU fallback exists)."""
import ctypes
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import rs_amd  # noqa: E402
from _util import (EXTRA_OPS, case, case_inputs, check_golden, extra_inputs, gen_info, manifest,  # noqa: E402
                   oracle_decode, oracle_encode)

pytestmark = pytest.mark.gpu

# Kernel variants. "auto" is the library default policy (XOR kernel for encode, generic then XOR kernel for
# repeated decode patterns): the only one this file runs. Release-library options (test_gpu_variants.py):
# jit = matrix-specialised bit-plane XOR kernel forced (rs_xj, hiprtc), v1jit = matrix-specialised
# nibble-table V = 1 kernel (rs_v1jit: the default for shapes the XOR kernel rejects), v1 / v1h = the generic
# V = 1 kernels (two / one nibble tables per input; v1h is the default generic kernel), cs_idx = the GF(2^16)
# route's syndromes on the gpr-indexed k_cs16 (the fallback of plans without threaded records).
# Diagnostic-library A/B families (DIAG_VARIANTS, librs_amd_diag.so): idx = LDS-DMA gpr-index kernel, table /
# mask = compiler-indexed reference kernels.
VARIANTS = {"jit": dict(jit=1), "v1jit": dict(jit=1, xj=0), "v1": dict(m8_mode=18, jit=0), "v1h": dict(m8_mode=20, jit=0), "idx": dict(m8_mode=2, jit=0),
            "table": dict(m8_mode=0, jit=0), "mask": dict(m8_mode=1, jit=0), "auto": dict(), "cs_idx": dict()}
DIAG_VARIANTS = ("idx", "table", "mask")
# codec options of a variant (set after construction): "cs_idx" runs the GF(2^16) route's syndromes on
# the gpr-indexed k_cs16 instead of the default threaded k_cs16t
VARIANT_OPTS = {"cs_idx": {"m16_cs_thread": 0}}


def lib_for(variant):
    """The rs_amd module of a variant's library (the diagnostic one for the A/B families)."""
    return rs_amd.diag_module() if variant in DIAG_VARIANTS else rs_amd


def codec_for(variant, k, r):
    c = lib_for(variant).Codec(k, r, **VARIANTS[variant])
    for name, value in VARIANT_OPTS.get(variant, {}).items():
        c.set_option(name, value)
    return c
CS_DEFAULT = "cs16t"  # rsg_last_kernel prefix of the default GF(2^16) syndrome kernel


def _pad(S):
    return (S + 15) // 16 * 16


def run_case_gpu(c, variant, options=None):
    k, r, S, n = c["k"], c["r"], c["S"], c["n"]
    P = _pad(S)
    host = np.zeros((n, k + r, P), np.uint8)
    er = None
    for s in range(n):
        buf, er = case_inputs(c, s)
        host[s, :, :S] = buf
    dev = torch.from_numpy(host).cuda()
    codec = codec_for(variant, k, r)
    for name, value in (options or {}).items():
        codec.set_option(name, value)
    st = torch.cuda.current_stream()
    base = dev.data_ptr()
    stride = (k + r) * P
    rc = 0
    if c["op"] in ("encode", "encode_iota", "gmatrix"):
        rc = codec.encode_raw(base, stride, P, base + k * P, stride, P, n, S, st)
        torch.cuda.synchronize()
        out = dev[:, k:, :S].cpu().numpy()
    else:
        if c["op"] == "decode":
            assert codec.encode_raw(base, stride, P, base + k * P, stride, P, n, S, st) == 0
            dev[:, torch.from_numpy(er)] = 0
        rc = codec.decode_raw(base, stride, P, n, S, er, st)
        torch.cuda.synchronize()
        out = dev[:, :, :S].cpu().numpy()
    return rc, out.tobytes(), codec.last_kernel, codec.subfield


GPU_CASES = [c["name"] for c in manifest()["cases"] if c["op"] not in EXTRA_OPS]
# odd symbol sizes are a drop-in API case (the reference's Release semantics); rsg_* rejects them
BATCH_CASES = [n for n in GPU_CASES if not n.startswith("odd_")]
EXTRA_CASES = [c["name"] for c in manifest()["cases"] if c["op"] in EXTRA_OPS]
# kernels (rsg_last_kernel) of the production GF(2^16) path over full 1 KiB column chunks
M16_PRODUCTION = ("apply_m16_v1", "apply_m16_rt16", "apply_m16_rt32")  # R <= 32: the compiled tiles


@pytest.mark.parametrize("name", BATCH_CASES)
def test_golden_batch_api(name):
    golden_batch_case(name, "auto")


def golden_batch_case(name, variant):
    c = case(name)
    m16 = c["k"] + c["r"] > 255 and c["op"] != "gmatrix"
    if variant not in ("auto", "cs_idx") and m16:
        pytest.skip("m = 16 code: the GF(256) kernel variants do not apply ('auto' and 'cs_idx' cover it)")
    if variant == "cs_idx" and not m16:
        pytest.skip("GF(256) code: no syndrome route")
    cs = "cs16" if variant == "cs_idx" else CS_DEFAULT
    rc, out, kern, m = run_case_gpu(c, variant)
    assert rc == c["rc"], (rc, kern)
    if name.startswith("c5_") and name.endswith(("_1k", "_2k")):  # full 1 KiB chunks: the production GF(2^16) path
        assert kern in M16_PRODUCTION or kern.startswith(cs + "+"), kern
    if name.startswith("max_n_route"):  # k + r = 65535 on whole 1 KiB columns
        # encode: the syndrome route; decode: a new pattern's first 64 MiB launch runs the dense plan
        # (m16_route_min_bytes), so the route is pinned by a second run that takes it at once
        assert kern.startswith(cs + "+") if c["op"] == "encode" else kern in M16_PRODUCTION, kern
        if c["op"] == "decode":
            rc2, out2, kern2, _ = run_case_gpu(c, variant, {"m16_route_min_bytes": 0})
            assert rc2 == c["rc"] and kern2.startswith(cs + "+bs16+xor+"), kern2  # the re-encode decode
            check_golden(c, out2)
    check_golden(c, out)


DROPIN = [n for n in GPU_CASES if n.startswith(("c1_", "kat_", "ex_", "edge_", "c2_", "m4_", "m8_", "odd_"))]


@pytest.mark.parametrize("name", DROPIN)
def test_golden_drop_in_api(name):
    """The reference-compatible per-call API (host symbol_seq_t in, host out)."""
    c = case(name)
    k, r, n = c["k"], c["r"], c["n"]
    rs = rs_amd.RS()
    outs, rc = [], 0
    for s in range(n):
        buf, er = case_inputs(c, s)
        syms = [np.ascontiguousarray(buf[i]) for i in range(k + r)]
        if c["op"] in ("encode", "encode_iota", "gmatrix"):
            rc = rs.generate_repair_symbols(syms[:k], syms[k:])
            outs.append(b"".join(x.tobytes() for x in syms[k:]))
        else:
            if c["op"] == "decode":
                assert rs.generate_repair_symbols(syms[:k], syms[k:]) == 0
                for i in np.nonzero(er)[0]:
                    syms[i][:] = 0
            rc = rs.restore_symbols(k, r, syms, er, c["t"])
            outs.append(b"".join(x.tobytes() for x in syms))
    rs.close()
    assert rc == c["rc"]
    check_golden(c, b"".join(outs))


@pytest.mark.parametrize("name", [n for n in DROPIN if n.startswith(("odd_", "ex_", "c1_", "c2_"))])
def test_golden_drop_in_seq_create(name):
    """The same golden cases on library-allocated sequences (seq_create: page-locked arena stripes at
    stride pad16(S), zero-copy launches or DMA in place), as the reference's callers allocate them
    (src/example.c, test_random_data.c); includes the odd symbol sizes."""
    c = case(name)
    k, r, n = c["k"], c["r"], c["n"]
    rs = rs_amd.RS()
    outs, rc = [], 0
    for s in range(n):
        buf, er = case_inputs(c, s)
        q = rs_amd.Seq(k + r, c["S"])
        for i in range(k + r):
            q.symbols[i][:] = buf[i]
        if c["op"] in ("encode", "encode_iota", "gmatrix"):
            rc = rs.generate_repair_symbols(q, r)
            outs.append(b"".join(x.tobytes() for x in q.symbols[k:]))
        else:
            if c["op"] == "decode":
                assert rs.generate_repair_symbols(q, r) == 0
                for i in np.nonzero(er)[0]:
                    q.symbols[i][:] = 0
            rc = rs.restore_symbols(k, r, q, er, c["t"])
            outs.append(b"".join(x.tobytes() for x in q.symbols))
        q.close()
    rs.close()
    assert rc == c["rc"]
    check_golden(c, b"".join(outs))


def test_config2_all_stripes_vs_oracle():
    config2_case("auto")


def config2_case(variant):
    """BASELINE config 2: k=10, r=4, 4 KiB symbols, 1024 stripes -- every stripe bit-exact vs the oracle."""
    k, r, S, n = 10, 4, 4096, 1024
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0xC2)
    codec = codec_for(variant, k, r)
    codec.encode(dev)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    want = got.copy()
    want[:, k:] = 0
    for s in range(n):
        assert np.array_equal(want[s, :k].reshape(-1), gen_info(0xC2, s, k * S))
        assert oracle_encode(k, r, want[s]) == 0
    assert np.array_equal(got, want)
    er = rs_amd.bench_pattern(k, r)
    dev[:, torch.from_numpy(er)] = 0
    codec.decode(dev, er)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), got)


def test_config3_shape_roundtrip():
    config3_case("auto")


def config3_case(variant):
    """k=128, r=32, 64 KiB symbols on 48 stripes: device generator == host generator, repair of sampled
    stripes == oracle, fingerprint of info unchanged after erase + restore, random patterns too."""
    k, r, S, n = 128, 32, 65536, 48
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0x5EED)
    codec = codec_for(variant, k, r)
    codec.encode(dev)
    fp0 = torch.zeros(n, dtype=torch.int64, device="cuda")
    rs_amd.fingerprint(dev, 0, k + r, fp0)
    torch.cuda.synchronize()
    for s in (0, n // 2, n - 1):
        host = dev[s].cpu().numpy()
        assert np.array_equal(host[:k].reshape(-1), gen_info(0x5EED, s, k * S))
        want = host.copy()
        want[k:] = 0
        assert oracle_encode(k, r, want) == 0
        assert np.array_equal(host, want), f"stripe {s}"
    rng = np.random.default_rng(3)
    patterns = [rs_amd.bench_pattern(k, r)]
    for t in (32, 17, 1):
        er = np.zeros(k + r, bool)
        er[rng.choice(k + r, t, replace=False)] = True
        patterns.append(er)
    for er in patterns:
        dev[:, torch.from_numpy(er)] = 0xA5  # poison: erased slots are never read
        codec.decode(dev, er)
        dev[:, torch.from_numpy(np.r_[np.zeros(k, bool), er[k:]])] = 0
        codec.encode(dev)  # re-derive the erased repair slots for the next pattern
        fp = torch.zeros(n, dtype=torch.int64, device="cuda")
        rs_amd.fingerprint(dev, 0, k + r, fp)
        torch.cuda.synchronize()
        assert torch.equal(fp, fp0), f"pattern t={int(er.sum())}"


def test_inflight_scalar_load_fix_on_the_kernels_run(tmp_path, monkeypatch):
    """GPUTEST_r04's illegal address: sload32 let the compiler put the base of its
    second s_load_dwordx16 inside the first one's destination. The kernels that inline it, at large grids:
    rs_v1jit at the faulting C2 launch (1024 stripes x 4 chunks) and at 128 x 64 (its default shape), and
    the per-stripe solve k_apply_m8_v1<0> over 2048 stripes -- bit-exact -- and the code objects the box
    compiled for them (fresh JIT cache) and the loaded release library pass scripts/isa_hazards.py."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import isa_hazards
    monkeypatch.setenv("RS_AMD_JIT_CACHE", str(tmp_path))
    for k, r, S, n in ((10, 4, 4096, 1024), (128, 64, 4096, 64)):
        dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
        rs_amd.fill_info(dev, k, seed=0x51)
        codec = rs_amd.Codec(k, r, jit=1, xj=0)
        codec.encode(dev)
        torch.cuda.synchronize()
        assert codec.last_kernel.startswith("rs_v1jit"), codec.last_kernel
        got = dev.cpu().numpy()
        for s in (0, n - 1):
            want = got[s].copy()
            want[k:] = 0
            assert oracle_encode(k, r, want) == 0
            assert np.array_equal(got[s], want), (k, r, s)
        er = rs_amd.bench_pattern(k, r)
        dev[:, torch.from_numpy(er)] = 0
        codec.decode(dev, er)
        torch.cuda.synchronize()
        assert codec.last_kernel.startswith("rs_v1jit"), codec.last_kernel
        assert np.array_equal(dev.cpu().numpy(), got), (k, r)
    # the per-stripe solve (k_apply_m8_v1<0>, re-encode route) over 2048 all-distinct stripes (the ring kernel
    # by option: the default solve is the prefetching k_apply_m8_pf)
    k, r, S, n = 128, 32, 2048, 2048
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0x52)
    codec = rs_amd.Codec(k, r, batch_plans=1)
    codec.set_option("m8_ps_kernel", 0)
    codec.encode(dev)
    torch.cuda.synchronize()
    full = dev.clone()
    rng = np.random.default_rng(52)
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        pats[s, rng.choice(k, r, replace=False)] = True
    dev[torch.from_numpy(pats).cuda()] = 0
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    assert codec.last_kernel.endswith("+apply_m8_v1_ps"), codec.last_kernel
    assert torch.equal(dev, full)
    objs = [os.path.join(tmp_path, f) for f in os.listdir(tmp_path) if f.startswith("v1_") and f.endswith(".co")]
    assert len(objs) >= 2, os.listdir(tmp_path)
    for path in objs + [rs_amd.LIB_PATH]:
        found = isa_hazards.hazards(isa_hazards.disassemble(path))
        assert not found, (path, found[:3])


def test_decode_matches_oracle_on_noncodewords():
    noncodeword_case(["auto"])


def noncodeword_case(variants):
    """Arbitrary (non-codeword) survivors: the GPU decoder applies exactly the reference's linear map."""
    k, r, S = 128, 32, 8192
    rng = np.random.default_rng(11)
    er = np.zeros(k + r, bool)
    er[rng.choice(k + r, 27, replace=False)] = True
    host = rng.integers(0, 256, (2, k + r, S), dtype=np.uint8)
    host[:, er] = 0
    dev = torch.from_numpy(host).cuda()
    for variant in variants:
        d = dev.clone()
        codec_for(variant, k, r).decode(d, er)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
        for s in range(2):
            want = host[s].copy()
            assert oracle_decode(k, r, want, er, int(er.sum())) == 0
            assert np.array_equal(got[s], want), variant


def test_errors():
    codec = rs_amd.Codec(4, 2)
    dev = torch.zeros((1, 6, 64), dtype=torch.uint8, device="cuda")
    er = np.array([1, 1, 1, 0, 0, 0], bool)
    assert codec.decode(dev, er, check=False) == rs_amd.RS_ERR_CANNOT_RESTORE
    assert codec.encode_raw(dev.data_ptr() + 1, 6 * 64, 64, dev.data_ptr() + 256, 6 * 64, 64, 1, 64,
                            torch.cuda.current_stream()) == rs_amd.RS_ERR_INVALID
    assert codec.encode_raw(dev.data_ptr(), 6 * 64, 64, dev.data_ptr() + 256, 6 * 64, 64, 1, 63,
                            torch.cuda.current_stream()) == rs_amd.RS_ERR_INVALID  # rsg_*: odd symbol size
    rs = rs_amd.RS()
    syms = [np.zeros(9, np.uint8) for _ in range(7)]
    assert rs.generate_repair_symbols(syms[:4], syms[4:7]) == 0  # drop-in: the reference's odd-size semantics
    assert rs.restore_symbols(4, 2, syms[:5], np.zeros(6, bool), 0) == rs_amd.RS_ERR_INVALID  # length != k + r


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (the box has one)")
def test_calls_keep_the_callers_current_device():
    """A codec on device 0 called from a thread whose current device is 1 (a host driving several GPUs, or
    torch code relying on its current device) leaves the thread on device 1: every public entry that selects
    the codec's device restores the caller's (rs_core.hpp CallerDevice)."""
    k, r, S, n = 10, 4, 4096, 4
    torch.cuda.set_device(1)
    try:
        dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda:0")
        rs_amd.fill_info(dev, k, seed=3)
        codec = rs_amd.Codec(k, r, device=0)
        assert torch.cuda.current_device() == 1
        codec.encode(dev)
        er = rs_amd.bench_pattern(k, r)
        codec.decode(dev, er)
        codec.decode_batch(dev, np.tile(er, (n, 1)))
        assert torch.cuda.current_device() == 1
        rs = rs_amd.RS()
        syms = [np.zeros(64, np.uint8) for _ in range(k + r)]
        assert rs.generate_repair_symbols(syms[:k], syms[k:]) == 0
        rs.close()
        assert torch.cuda.current_device() == 1
        codec.close()
    finally:
        torch.cuda.set_device(0)


def test_fingerprint_matches_cpu_port():
    """The device fingerprint used by bench.py's verification == tests/_util.py:fingerprint_np."""
    from _util import fingerprint_np
    k, r, S, n = 10, 4, 4096, 5
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0xF1, stripe0=7)
    rs_amd.Codec(k, r).encode(dev)
    fp = torch.zeros(n, dtype=torch.int64, device="cuda")
    rs_amd.fingerprint(dev, 0, k + r, fp)
    torch.cuda.synchronize()
    host = dev.cpu().numpy()
    for s in range(n):
        assert np.array_equal(host[s, :k].reshape(-1), gen_info(0xF1, 7 + s, k * S))
        assert int(fp[s]) == fingerprint_np(host[s], 0, k + r)


@pytest.mark.parametrize("plans,n", [(0, 40), (1, 40), (2, 40), (2, 100)])
@pytest.mark.parametrize("S", [8192, 8712])
def test_decode_batch_per_stripe_patterns(S, plans, n):
    """rsg_decode_batch: every stripe has its own erasure pattern (information and repair erasures,
    stripes with nothing to restore, repeated patterns) -- each stripe bit-exact vs the oracle, with
    host plans per pattern (0), device-built plans (1) and the default (2: 11 distinct patterns at
    n = 40 take host plans; 23 at n = 100 pass the 16-pattern threshold, where grouping stops and the
    device plans take over); S = 8712 adds tail columns."""
    k, r = 128, 32
    rng = np.random.default_rng(21)
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0xB7)
    codec = rs_amd.Codec(k, r, batch_plans=plans)
    codec.encode(dev)
    torch.cuda.synchronize()
    full = dev.cpu().numpy()
    shared = [rng.choice(k + r, t, replace=False) for t in (32, 5, 17)]
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        m = s % 5
        if m < 3:
            pats[s, shared[m]] = True  # repeated patterns (one launch each)
        elif m == 3:
            pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True  # unique
        else:
            pats[s, k + rng.choice(r, 3, replace=False)] = True  # repair-only: nothing to restore
    poisoned = full.copy()
    poisoned[pats] = 0
    dev.copy_(torch.from_numpy(poisoned))
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    if plans == 2:
        lk = codec.last_kernel
        assert ("apply_m8_v1_ps" in lk or "apply_m8_pf" in lk) == (n == 100), lk
    got = dev.cpu().numpy()
    for s in range(n):
        want = poisoned[s].copy()
        assert oracle_decode(k, r, want, pats[s], int(pats[s].sum())) == 0
        assert np.array_equal(got[s], want), f"stripe {s}"
        assert np.array_equal(got[s, :k], full[s, :k])
    # one stripe beyond r erasures: nothing is written, RS_ERR_CANNOT_RESTORE
    bad = pats.copy()
    bad[7, :] = False
    bad[7, : r + 1] = True
    before = dev.clone()
    assert codec.decode_batch(dev, bad, check=False) == rs_amd.RS_ERR_CANNOT_RESTORE
    torch.cuda.synchronize()
    assert torch.equal(dev, before)


@pytest.mark.parametrize("S", [2048, 11008])
def test_xor_kernel_with_tail_columns(S):
    """Symbols that are not a multiple of the 2 KiB column block: the XOR kernel covers the full blocks,
    the generic tail kernel the rest -- encode and decode bit-exact vs the oracle."""
    k, r, n = 128, 32, 3
    rng = np.random.default_rng(S)
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    codec = rs_amd.Codec(k, r, jit=1)
    codec.encode(dev)
    torch.cuda.synchronize()
    assert codec.last_kernel.startswith("rs_xj")
    got = dev.cpu().numpy()
    for s in range(n):
        want = host[s].copy()
        assert oracle_encode(k, r, want) == 0
        assert np.array_equal(got[s], want), f"encode stripe {s}"
    er = np.zeros(k + r, bool)
    er[rng.choice(np.r_[0:3, 4:k + r], 28, replace=False)] = True
    er[3] = True  # 29 erasures, at least one information symbol
    dev[:, torch.from_numpy(er)] = 0
    codec.decode(dev, er)
    torch.cuda.synchronize()
    back = dev.cpu().numpy()
    assert codec.last_kernel.startswith("rs_xj")
    for s in range(n):
        want = got[s].copy()
        want[er] = 0
        assert oracle_decode(k, r, want, er, int(er.sum())) == 0
        assert np.array_equal(back[s], want), f"decode stripe {s}"


@pytest.mark.parametrize("k,r,S,n", [(128, 32, 4096 + 1032, 96), (10, 4, 1024 + 8, 300), (200, 55, 2048, 24)])
def test_decode_batch_device_plans_distinct_patterns(k, r, S, n):
    """Every stripe lost a different random set (1..r symbols, information and repair slots): the
    default policy builds the decode matrices on the device; every stripe is bit-exact vs the oracle
    and the information symbols come back."""
    rng = np.random.default_rng(k * 7 + n)
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0xC3)
    codec = rs_amd.Codec(k, r)
    codec.encode(dev)
    torch.cuda.synchronize()
    full = dev.cpu().numpy()
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    pats[0, :] = False
    pats[0, :r] = True  # r information erasures (largest plan)
    poisoned = full.copy()
    poisoned[pats] = 0
    dev.copy_(torch.from_numpy(poisoned))
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    assert codec.last_kernel == "apply_m8_v1_ps"
    got = dev.cpu().numpy()
    for s in range(n):
        assert np.array_equal(got[s, :k], full[s, :k]), f"stripe {s}"
        if s % 8 == 0:
            want = poisoned[s].copy()
            assert oracle_decode(k, r, want, pats[s], int(pats[s].sum())) == 0
            assert np.array_equal(got[s], want), f"stripe {s}"


@pytest.mark.parametrize("k,r,S,n", [(300, 200, 1024 + 8, 40), (4096, 1024, 1024, 24)])
def test_decode_batch_m16_stream_plans(k, r, S, n):
    """GF(2^16) codes with more than 16 distinct patterns in one rsg_decode_batch: the codec's batch plan
    is rebuilt on the stream for every pattern (k_plan16_*). Information symbols come back on every
    stripe (64-row asm tiles and the compiled kernel for R <= 32, split-K single-stripe launches,
    repair-only stripes skipped); stripes bit-exact vs the oracle where it is quick, and the whole
    batch byte-identical to the cached per-pattern plans (batch_plans=0)."""
    rng = np.random.default_rng(k + n)
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0xD5)
    codec = rs_amd.Codec(k, r)
    codec.encode(dev)
    torch.cuda.synchronize()
    full = dev.cpu().numpy()
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        if s % 7 == 6:
            pats[s, k + rng.choice(r, 3, replace=False)] = True  # repair-only: nothing to restore
        else:
            pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    pats[0, :] = False
    pats[0, :r] = True  # r information erasures (largest plan)
    pats[1, :] = False
    pats[1, rng.choice(k, 20, replace=False)] = True  # R <= 32 (compiled kernel tiles)
    poisoned = full.copy()
    poisoned[pats] = 0
    dev.copy_(torch.from_numpy(poisoned))
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    for s in range(n):
        assert np.array_equal(got[s, :k], full[s, :k]), f"stripe {s}"
    for s in range(n) if k + r <= 1024 else (0, 1, 2, 5, 6):  # C5: a sample (the oracle takes ~1 s a stripe)
        want = poisoned[s].copy()
        assert oracle_decode(k, r, want, pats[s], int(pats[s].sum())) == 0
        assert np.array_equal(got[s], want), f"stripe {s}"
    dev.copy_(torch.from_numpy(poisoned))
    assert rs_amd.Codec(k, r, batch_plans=0).decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), got)


def ps16_kernel_ok(name, ps):
    """rsg_last_kernel of the per-stripe GF(2^16) route: syndromes (m16_ps 1) or the re-encode variant (2)."""
    if ps == 2:
        return name.startswith("ps16r+") and name.endswith("+xor+apply_m16_v1_ps")
    return name == f"ps16+{CS_DEFAULT}+apply_m16_v1_ps"


@pytest.mark.parametrize("ps", [1, 2])
def test_decode_batch_m16_per_stripe_route_vs_golden(ps):
    """rsg_decode_batch at C5 with a different pattern on every stripe (reference reed_solomon.c:443-559):
    the per-stripe GF(2^16) route (ps 1: one syndrome pass over all k + r slots, then each stripe's own
    device-built t_info x t solve; ps 2: the encode route over the information slots + the received repair
    rows, then each stripe's t_info x t_info Cauchy solve). Every stripe's output equals the reference golden
    of its pattern; erased information slots hold garbage on input; a repair-only stripe and a stripe without
    erasures are left untouched."""
    cases = [case(nm) for nm in GPU_CASES if nm.startswith("c5ps_")]
    assert len(cases) >= 8
    k, r, S = 4096, 1024, 1024
    buf0, _ = case_inputs(cases[0], 0)
    n = len(cases) + 2
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    dev[:, :k] = torch.from_numpy(buf0[:k]).cuda()
    codec = rs_amd.Codec(k, r)
    codec.set_option("m16_ps", ps)
    codec.encode(dev)
    torch.cuda.synchronize()
    full = dev.cpu().numpy()
    pats = np.zeros((n, k + r), bool)
    for s, c in enumerate(cases):
        pats[s, c["erased"]] = True
    pats[len(cases), k + np.arange(5)] = True  # repair-only: nothing to restore
    rng = np.random.default_rng(5)
    host = full.copy()
    host[pats] = 0
    info_er = pats.copy()
    info_er[:, k:] = False
    host[info_er] = rng.integers(0, 256, (int(info_er.sum()), S), dtype=np.uint8)  # garbage: zeroed first
    dev.copy_(torch.from_numpy(host))
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    assert ps16_kernel_ok(codec.last_kernel, ps), codec.last_kernel
    got = dev.cpu().numpy()
    for s, c in enumerate(cases):
        check_golden(c, got[s].tobytes())
    assert np.array_equal(got[len(cases)], host[len(cases)])
    assert np.array_equal(got[-1], full[-1])


@pytest.mark.parametrize("ps", [1, 2, 3])
@pytest.mark.parametrize("k,r,S,n", [(1000, 200, 2048, 37), (300, 64, 1024, 70), (600, 100, 3072, 5)])
def test_decode_batch_m16_per_stripe_route(k, r, S, n, ps):
    """The per-stripe GF(2^16) route (ps 1 syndromes, 2 re-encode, 3 the default choice: re-encode when the
    batch's largest pattern needs >= 13/16 r syndromes) on assorted shapes: random patterns of 1..r erasures
    anywhere (garbage in erased slots), against the oracle on a sample and byte-identical to the
    per-pattern plans (m16_ps = 0); erased repair slots keep what they held."""
    rng = np.random.default_rng(k + r + n)
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0xE1)
    codec = rs_amd.Codec(k, r)
    codec.set_option("m16_ps", ps)
    codec.encode(dev)
    torch.cuda.synchronize()
    full = dev.cpu().numpy()
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    pats[0, :] = False
    pats[0, :r] = True  # r information erasures
    host = full.copy()
    host[pats] = rng.integers(0, 256, (int(pats.sum()), S), dtype=np.uint8)
    dev.copy_(torch.from_numpy(host))
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    D = min(r, (int(pats.sum(1).max()) + 31) // 32 * 32)
    assert ps16_kernel_ok(codec.last_kernel, ps if ps < 3 else (2 if 16 * D >= 13 * r else 1)), codec.last_kernel
    got = dev.cpu().numpy()
    assert np.array_equal(got[:, :k], full[:, :k])
    rep = pats.copy()
    rep[:, :k] = False
    assert np.array_equal(got[rep], host[rep])  # erased repair slots not written
    for s in list(range(0, n, max(1, n // 5))) + [n - 1]:
        want = host[s].copy()
        want[pats[s]] = 0
        assert oracle_decode(k, r, want, pats[s], int(pats[s].sum())) == 0
        assert np.array_equal(got[s, :k], want[:k]), f"stripe {s}"
    old = rs_amd.Codec(k, r)
    old.set_option("m16_ps", 0)
    dev.copy_(torch.from_numpy(host))
    assert old.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    assert old.last_kernel != codec.last_kernel
    assert np.array_equal(dev.cpu().numpy()[:, :k], got[:, :k])


def test_decode_batch_m16_per_stripe_reenc_falls_back():
    """m16_ps 2 needs the codec's encode on the GF(2^16) route (k >= 64 inputs): a code with k = 40 (k + r >
    255) encodes densely, so its per-stripe batches take the syndrome route -- bit-exact vs the oracle."""
    k, r, S, n = 40, 230, 1024, 6
    rng = np.random.default_rng(40)
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0x40)
    codec = rs_amd.Codec(k, r)
    codec.set_option("m16_ps", 2)
    codec.encode(dev)
    torch.cuda.synchronize()
    full = dev.cpu().numpy()
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    host = full.copy()
    host[pats] = rng.integers(0, 256, (int(pats.sum()), S), dtype=np.uint8)
    dev.copy_(torch.from_numpy(host))
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    assert ps16_kernel_ok(codec.last_kernel, 1), codec.last_kernel
    got = dev.cpu().numpy()
    assert np.array_equal(got[:, :k], full[:, :k])
    for s in range(n):
        want = host[s].copy()
        want[pats[s]] = 0
        assert oracle_decode(k, r, want, pats[s], int(pats[s].sum())) == 0
        assert np.array_equal(got[s, :k], want[:k]), f"stripe {s}"


@pytest.mark.parametrize("ps,overlap", [(1, 0), (1, 1), (2, 0)])
@pytest.mark.parametrize("chunk", [1, 3, 7])
def test_decode_batch_m16_per_stripe_route_chunks(chunk, ps, overlap):
    """The per-stripe route in several chunks (m16_ps_chunk): double-buffered plans, and with m16_ps_overlap
    the next chunk's syndrome pass on its own stream into the other syndrome buffer (ps 2: the re-encode
    variant, whose fixed pass covers each chunk's stripe range); byte-identical to the one-chunk decode,
    stripes without erased information (skipped) mixed in."""
    k, r, S, n = 700, 120, 1024, 17
    rng = np.random.default_rng(chunk * 10 + overlap)
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0xC4)
    one = rs_amd.Codec(k, r)
    one.encode(dev)
    torch.cuda.synchronize()
    full = dev.cpu().numpy()
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    pats[2, :] = False
    pats[2, k:k + 5] = True  # repair erasures only: not restored, not in the chunks
    host = full.copy()
    host[pats] = rng.integers(0, 256, (int(pats.sum()), S), dtype=np.uint8)
    dev.copy_(torch.from_numpy(host))
    assert one.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    want = dev.cpu().numpy()
    assert np.array_equal(want[:, :k], full[:, :k])
    cdc = rs_amd.Codec(k, r)
    cdc.set_option("m16_ps", ps)
    cdc.set_option("m16_ps_chunk", chunk)
    cdc.set_option("m16_ps_overlap", overlap)
    for it in range(3):  # the second call reuses the streams, events and buffers; the third regrows them
        if it == 2:
            cdc.trim()
        dev.copy_(torch.from_numpy(host))
        assert cdc.decode_batch(dev, pats) == 0
        torch.cuda.synchronize()
        assert ps16_kernel_ok(cdc.last_kernel, ps), cdc.last_kernel
        assert np.array_equal(dev.cpu().numpy(), want)


SYN_ROUTE_SHAPES = [(128, 32, 8192, 64), (10, 4, 4096, 300), (30, 17, 2048, 40), (128, 32, 32768, 1030),
                    (20, 9, 4096 + 520, 33), (60, 40, 4096, 50)]


# release-library settings: the three routes, the prefetching solve (10, the default) and the LDS-ring solve
# with two or one nibble tables per input
# (the A/B kernels, overlapped chunks and multi-chunk workgroups: tests/test_gpu_variants.py, diagnostic library)
@pytest.mark.parametrize("route,ovl,kern,cpb", [(2, 0, 0, 1), (1, 0, 0, 1), (0, 0, 0, 1), (2, 0, 3, 1), (1, 0, 3, 1),
                                                (0, 0, 3, 1), (2, 0, 10, 1), (1, 0, 10, 1), (0, 0, 10, 1)])
@pytest.mark.parametrize("k,r,S,n", SYN_ROUTE_SHAPES)
def test_decode_batch_syndrome_route(k, r, S, n, route, ovl, kern, cpb):
    syndrome_route_case(rs_amd, k, r, S, n, route, ovl, kern, cpb)


@pytest.mark.parametrize("kern", [0, 10])
@pytest.mark.parametrize("route", [1, 2])
@pytest.mark.parametrize("k,r,S,n", [SYN_ROUTE_SHAPES[0], SYN_ROUTE_SHAPES[2], SYN_ROUTE_SHAPES[5]])
def test_decode_batch_syndrome_route_unmasked(k, r, S, n, route, kern):
    """Option m8_syn_masked 0: the plain fixed pass over the slots as they are (garbage in the erased ones) and
    a solve that XORs g + c into the erased information slots."""
    syndrome_route_case(rs_amd, k, r, S, n, route, 0, kern, 1, masked=0)



def syndrome_route_case(lib, k, r, S, n, route, ovl, kern, cpb, masked=1, coord=0):
    """Device-built per-stripe decodes through the syndrome route (route 1: r syndromes of every slot on
    the XOR kernel, then each stripe's t_info x t solve XORed into the erased slots, which are not zeroed
    first; route 2: the re-encode differences [G | I] of every slot, then a t_info x t_info Cauchy-inverse
    solve from the first t_info surviving repair rows; ovl 1: chunk i + 1's plans and syndromes on the codec's second stream beside chunk i's solve)
    and the survivor-matrix route (0). Erased slots hold garbage, not zeros: information slots come back
    bit-exact vs the oracle (which reads erased slots as zero), erased repair slots are left as they
    were. n = 1030 at 32 KiB spans two chunks of the syndrome scratch (and several overlapped ones).
    kern 1 / 2: the per-stripe solves on k_apply_m8_ps_w / _w2 (one / two dwords per lane) instead of the
    LDS-ring kernel; 3: the ring kernel with one nibble table per input (k_apply_m8_v1<2>); 9 / 10 / 11: the
    prefetching solve k_apply_m8_pf<1> / <2> / <3> (two / one nibble tables / one table with the multiples read
    from LDS) on packed records (route 0 keeps the ring kernel: survivor plans are not packed;
    r = 40 gives two output tiles and up to 40 inputs per stripe). cpb > 1: the
    ring kernel walks that many 1 KiB column chunks per workgroup (k_apply_m8_v1<6>; 64 > chunks per symbol). S = 4096 + 520 (survivor route only: the syndrome route needs whole 2 KiB columns)
    ends in a partial column chunk."""
    if route and S % 2048:
        pytest.skip("the syndrome route covers whole 2 KiB columns (other sizes take the survivor route)")
    rng = np.random.default_rng(k + 3 * n + route)
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(dev, k, seed=0xD5)
    codec = lib.Codec(k, r, batch_plans=1)
    codec.set_option("syn_route", route)
    codec.set_option("m8_syn_overlap", ovl)
    codec.set_option("m8_ps_kernel", kern)  # 1: the ring-free per-stripe solve kernel (k_apply_m8_ps_w)
    codec.set_option("m8_ps_cpb", cpb)
    codec.set_option("m8_syn_masked", masked)
    if coord:
        codec.set_option("m8_syn_coord", coord)
    codec.encode(dev)
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    pats[0, :] = False
    pats[0, :r] = True  # r information erasures
    pats[1, :] = False
    pats[1, k:] = True  # repair slots only: nothing to restore
    full = dev.clone()
    mask = torch.from_numpy(pats).cuda()
    garbage = torch.randint(0, 256, (int(pats.sum()), S), dtype=torch.uint8, device="cuda")
    dev[mask] = garbage
    poisoned = dev.clone()
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    fixed = {1: "syn_xj", 2: "reenc_xj"}.get(route)
    solve = "+apply_m8_pf" if kern >= 9 and S % 1024 == 0 else "+apply_m8_v1_ps"
    assert codec.last_kernel == ("apply_m8_v1_ps" if not route else
                                 fixed + solve + ("(overlap)" if ovl else "")), codec.last_kernel
    assert torch.equal(dev[:, :k], full[:, :k])
    rep_er = mask.clone()
    rep_er[:, :k] = False
    assert torch.equal(dev[rep_er], poisoned[rep_er])  # erased repair slots not written
    assert torch.equal(dev[:, k:][~mask[:, k:]], full[:, k:][~mask[:, k:]])
    for s in list(range(0, n, max(1, n // 6))) + [n - 1]:
        want = poisoned[s].cpu().numpy()
        want[pats[s]] = 0
        assert oracle_decode(k, r, want, pats[s], int(pats[s].sum())) == 0
        assert np.array_equal(dev[s, :k].cpu().numpy(), want[:k]), f"stripe {s}"


@pytest.mark.parametrize("plans", [0, 1])
@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("S", [2048, 2048 + 264])
def test_m16_kernels_vs_oracle(S, mode, plans):
    """GF(2^16) code with r > 32 (64-row tiles): the hand-scheduled kernel (m16_mode 0, tail columns
    by the compiled kernel) and the compiled kernel (2), with plans built on the host (m16_plans 0) or
    on the device (1), encode and decode, bit-exact vs the oracle."""
    k, r, n = 300, 200, 3
    rng = np.random.default_rng(S + mode)
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    codec = rs_amd.Codec(k, r)
    codec.set_option("m16_route", 0)  # the dense kernels under test (the syndrome route has its own tests)
    codec.set_option("m16_mode", mode)
    codec.set_option("m16_plans", plans)  # rebuilds the encode plan
    assert codec.subfield == 16
    codec.encode(dev)
    torch.cuda.synchronize()
    assert codec.last_kernel == ("apply_m16_v1" if mode == 0 else "apply_m16_rt64")
    got = dev.cpu().numpy()
    want = host.copy()
    for s in range(n):
        assert oracle_encode(k, r, want[s]) == 0
    assert np.array_equal(got, want)
    er = np.zeros(k + r, bool)
    er[rng.choice(k + r, r, replace=False)] = True
    er[:7] = True
    er[np.nonzero(er)[0][r:]] = False  # exactly r erasures, information slots 0..6 among them
    poisoned = got.copy()
    poisoned[:, er] = 0
    dev.copy_(torch.from_numpy(poisoned))
    codec.decode(dev, er)
    torch.cuda.synchronize()
    out = dev.cpu().numpy()
    for s in range(n):
        ref = poisoned[s].copy()
        assert oracle_decode(k, r, ref, er, int(er.sum())) == 0
        assert np.array_equal(out[s], ref)
        assert np.array_equal(out[s, :k], got[s, :k])


@pytest.mark.parametrize("plans", [0, 1])
def test_decode_batch_back_to_back_streams(plans):
    """Two rsg_decode_batch calls issued back to back on different streams (the second call reuses
    the codec's device scratch while the first may still run): both batches restore bit-exactly."""
    k, r, S, n = 128, 32, 8192, 48
    rng = np.random.default_rng(33 + plans)
    codec = rs_amd.Codec(k, r, batch_plans=plans)
    bufs, fulls, pats = [], [], []
    for b in range(2):
        dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
        rs_amd.fill_info(dev, k, seed=0x51 + b)
        codec.encode(dev)
        torch.cuda.synchronize()
        full = dev.cpu().numpy()
        pat = np.zeros((n, k + r), bool)
        for s in range(n):
            pat[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
        poisoned = full.copy()
        poisoned[pat] = 0
        dev.copy_(torch.from_numpy(poisoned))
        bufs.append(dev)
        fulls.append(full)
        pats.append(pat)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for b in range(2):
        assert codec.decode_batch(bufs[b], pats[b], stream=streams[b]) == 0
    torch.cuda.synchronize()
    for b in range(2):
        got = bufs[b].cpu().numpy()
        assert np.array_equal(got[:, :k], fulls[b][:, :k]), f"batch {b}"


@pytest.mark.parametrize("name", ["c5_dec_bench_1k", "c5_dec_bench_1k_n2", "c5_dec_info1000_1k_n2", "c5_dec_mixed_1k_n2"])
def test_c5_bench_decode_kernels_vs_golden(name):
    """The C5 bench decode's kernels (reference reed_solomon.c:443-559) pinned to the reference goldens at
    full 1 KiB chunks, n = 1 and n = 2 stripes: with m16_route_min_bytes = 0 the first launch takes the
    route -- for the bench pattern (closed under x -> x^16) the plain syndrome route with the k_bs16
    second stage over row orbits of 4; for other information-only patterns with t >= 0.9 r the
    re-encode decode (encode route over the surviving information + repair XOR + D_Rep); the plain
    route with the dense second stage for patterns with repair erasures."""
    c = case(name)
    rc, out, kern, m = run_case_gpu(c, "auto", {"m16_route_min_bytes": 0})
    assert rc == c["rc"] == 0 and m == 16
    if "bench" in name:  # erased set closed under x -> x^16: the plain route with the k_bs16 second stage
        assert kern == CS_DEFAULT + "+bs16", kern
    elif any(e >= c["k"] for e in c["erased"]):
        assert kern.startswith(CS_DEFAULT + "+apply"), kern
    else:
        assert kern.startswith(CS_DEFAULT + "+bs16+xor+"), kern
    check_golden(c, out)


@pytest.mark.parametrize("k,r,S,n", [(1000, 200, 2048, 12), (4096, 1024, 1024, 2), (300, 64, 3072, 9)])
def test_cs16_threaded_matches_indexed(k, r, S, n):
    """The threaded syndrome kernel k_cs16t (default) and the gpr-indexed k_cs16 (m16_cs_thread = 0) give
    byte-identical repair symbols, and byte-identical restores for the bench pattern, a random information
    pattern and a mixed pattern on the route (m16_route_min_bytes = 0); the restores equal the encoded
    stripes and stripe 0's repair equals the oracle's."""
    outs = {}
    for thr in (1, 0):
        dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
        rs_amd.fill_info(dev, k, seed=0xC516)
        codec = rs_amd.Codec(k, r)
        codec.set_option("m16_cs_thread", thr)
        codec.set_option("m16_route_min_bytes", 0)
        codec.encode(dev)
        torch.cuda.synchronize()
        assert codec.last_kernel.startswith("cs16t+" if thr else "cs16+"), codec.last_kernel
        full = dev.cpu().numpy()
        res = [full[:, k:].copy()]
        pats = [rs_amd.bench_pattern(k, r), np.zeros(k + r, bool), np.zeros(k + r, bool)]
        pats[1][np.random.default_rng(k).choice(k, r, replace=False)] = True
        pats[2][np.random.default_rng(r).choice(k + r, r, replace=False)] = True
        for er in pats:
            dev.copy_(torch.from_numpy(full))
            dev[:, torch.from_numpy(er)] = 0
            assert codec.decode(dev, er) == 0
            torch.cuda.synchronize()
            assert codec.last_kernel.split("+")[0] == ("cs16t" if thr else "cs16"), codec.last_kernel
            got = dev.cpu().numpy()
            assert np.array_equal(got[:, :k], full[:, :k]), codec.last_kernel
            res.append(got[:, :k].copy())
        outs[thr] = (full, res)
    for a, b in zip(outs[1][1], outs[0][1]):
        assert np.array_equal(a, b)
    if k + r <= 1500:
        want = outs[1][0][0].copy()
        assert oracle_encode(k, r, want) == 0
        assert np.array_equal(outs[1][0][0, k:], want[k:])


def cs16_overlapped_case(k, r, S, n):
    """m16_cs_overlap = 1 (off by default): the one-pattern syndrome route in four chunks with each chunk's syndromes
    on the codec's syndrome stream beside the previous chunk's second stage (two syndrome buffers) gives
    the same repair symbols and restores as the serial route (0, default), for the bench pattern (k_bs16 second
    stage), a random information pattern and a mixed pattern (dense second stage); twice per codec."""
    outs = {}
    for ovl in (1, 0):
        dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
        rs_amd.fill_info(dev, k, seed=0x0C5)
        codec = (rs_amd.diag_module() if ovl else rs_amd).Codec(k, r)  # overlap: a diagnostic-build option
        codec.set_option("m16_cs_overlap", ovl)
        codec.set_option("m16_route_min_bytes", 0)
        res = []
        for _ in range(2):
            dev[:, k:] = 0
            codec.encode(dev)
            torch.cuda.synchronize()
            assert codec.last_kernel.startswith(CS_DEFAULT + "+"), codec.last_kernel
            full = dev.cpu().numpy()
            res.append(full[:, k:].copy())
            pats = [rs_amd.bench_pattern(k, r), np.zeros(k + r, bool), np.zeros(k + r, bool)]
            pats[1][np.random.default_rng(k).choice(k, r, replace=False)] = True
            pats[2][np.random.default_rng(r).choice(k + r, r, replace=False)] = True
            for er in pats:
                dev.copy_(torch.from_numpy(full))
                dev[:, torch.from_numpy(er)] = 0
                assert codec.decode(dev, er) == 0
                torch.cuda.synchronize()
                got = dev.cpu().numpy()
                assert np.array_equal(got[:, :k], full[:, :k]), (ovl, codec.last_kernel)
                res.append(got.copy())
        outs[ovl] = (full, res)
    for a, b in zip(outs[1][1], outs[0][1]):
        assert np.array_equal(a, b)
    want = outs[1][0][n - 1].copy()
    assert oracle_encode(k, r, want) == 0
    assert np.array_equal(outs[1][0][n - 1, k:], want[k:])


def test_m16_route_encode_then_decode_on_two_streams():
    """A GF(2^16) route encode on stream A and a route decode on stream B issued back to back with one
    codec: the decode rewrites the codec's slot-offset scratch (d_goff) that A's k_cs16 may still be
    reading, so it must wait for A first. Both results bit-exact vs the oracle."""
    k, r, S, n = 1000, 200, 4096, 48
    rng = np.random.default_rng(4242)
    codec = rs_amd.Codec(k, r)
    a = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(a, k, seed=0x77)
    b = torch.zeros((2, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(b, k, seed=0x78)
    codec.encode(b)
    torch.cuda.synchronize()
    full_b = b.cpu().numpy()
    er = np.zeros(k + r, bool)
    er[rng.choice(k + r, 40, replace=False)] = True  # t <= 64: the route at once
    poisoned = full_b.copy()
    poisoned[:, er] = 0
    want_b = full_b.copy()
    want_b[:, k:][:, er[k:]] = 0  # erased repair slots are not restored
    b.copy_(torch.from_numpy(poisoned))
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        codec.encode(a, stream=sa)
        assert codec.last_kernel.startswith(CS_DEFAULT + "+"), codec.last_kernel
        codec.decode(b, er, stream=sb)
        assert codec.last_kernel.startswith(CS_DEFAULT + "+"), codec.last_kernel
        torch.cuda.synchronize()
        assert np.array_equal(b.cpu().numpy(), want_b)
        b.copy_(torch.from_numpy(poisoned))
        torch.cuda.synchronize()
    got = a.cpu().numpy()
    for s in (0, n // 2, n - 1):
        want = got[s].copy()
        want[k:] = 0
        assert oracle_encode(k, r, want) == 0
        assert np.array_equal(got[s], want), f"stripe {s}"


XJ_SHAPES = [(1, 1), (2, 1), (3, 16), (7, 17), (9, 5), (16, 8), (33, 31), (50, 33), (64, 48), (100, 60), (120, 51),
             (180, 34), (24, 200), (12, 243)]


@pytest.mark.parametrize("k,r", XJ_SHAPES)
def test_xor_kernel_shapes_vs_oracle(k, r):
    """The generated bit-plane XOR kernel (forced with jit=1) over assorted (k, r) with k + r <= 255 --
    one output, 16/17 outputs (role boundary), several roles, k not a multiple of 8, symbol sizes with
    tail columns -- encode and a random-erasure decode bit-exact vs the oracle."""
    rng = np.random.default_rng(k * 1000 + r)
    S = 2048 * int(rng.integers(1, 3)) + 8 * int(rng.integers(0, 200))
    n = 2
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    codec = rs_amd.Codec(k, r, jit=1)
    codec.encode(dev)
    torch.cuda.synchronize()
    n_src = ctypes.c_size_t()
    eligible = rs_amd._lib.rsg_xj_source(k, r, None, 0, None, 0, ctypes.byref(n_src)) == 0
    assert codec.last_kernel.startswith("rs_xj" if eligible else "rs_v1jit"), codec.last_kernel
    got = dev.cpu().numpy()
    want = host.copy()
    for s in range(n):
        assert oracle_encode(k, r, want[s]) == 0
    assert np.array_equal(got, want)
    er = np.zeros(k + r, bool)
    t = int(rng.integers(1, r + 1))
    er[rng.choice(k + r, t, replace=False)] = True
    if not er[:k].any():
        er[rng.integers(0, k)] = True
        er[np.nonzero(er[k:])[0][0] + k] = False
    poisoned = got.copy()
    poisoned[:, er] = 0
    dev.copy_(torch.from_numpy(poisoned))
    codec.decode(dev, er)
    torch.cuda.synchronize()
    out = dev.cpu().numpy()
    for s in range(n):
        ref = poisoned[s].copy()
        assert oracle_decode(k, r, ref, er, int(er.sum())) == 0
        assert np.array_equal(out[s], ref), f"stripe {s}"


@pytest.mark.parametrize("k,r,S", [(250, 33, 1024), (300, 64, 2048 + 40), (200, 65, 1024 + 1000), (1000, 100, 2048),
                                   (400, 129, 3072 + 4), (2000, 100, 1024)])
@pytest.mark.parametrize("route,col", [(0, 256), (1, 256)])
def test_m16_kernel_shapes_vs_oracle(k, r, S, route, col):
    m16_shapes_case(rs_amd, k, r, S, route, col)


def m16_shapes_case(lib, k, r, S, route, col):
    """GF(2^16) codes around the 64-row tiles of k_apply_m16_v1 (one partial tile, exactly one tile, a
    1-row second tile, three tiles) with tail columns, encode and decode bit-exact vs the oracle. Two
    stripes make small grids, so every case also runs split-K (k=2000: 31 input slices). Route 0: the
    dense kernel; route 1: the syndrome route where it applies (K >= 64, whole 1 KiB chunks; other
    launches of a route plan fall back to its dense plan); col: the route kernels' block layout
    (option m16_cs_col, 1 KiB column per tile or 4 tiles per 256-byte column)."""
    rng = np.random.default_rng(k + 7 * r + S)
    n = 2
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    codec = lib.Codec(k, r)
    codec.set_option("m16_route", route)
    codec.set_option("m16_route_min_bytes", 0)  # decode patterns on the route from their first launch
    codec.set_option("m16_cs_col", col)
    assert codec.subfield == 16
    codec.encode(dev)
    torch.cuda.synchronize()
    routed = route == 1 and k >= 64 and S % 1024 == 0
    dense = "apply_m16_v1" if r > 32 else f"apply_m16_rt{16 if r <= 16 else 32}"
    assert codec.last_kernel == (CS_DEFAULT + "+bs16" if routed else dense), codec.last_kernel
    got = dev.cpu().numpy()
    want = host.copy()
    for s in range(n):
        assert oracle_encode(k, r, want[s]) == 0
    assert np.array_equal(got, want)
    er = np.zeros(k + r, bool)
    er[rng.choice(k, min(k, r), replace=False)] = True  # r information erasures: the largest decode
    poisoned = got.copy()
    poisoned[:, er] = 0
    dev.copy_(torch.from_numpy(poisoned))
    codec.decode(dev, er)
    torch.cuda.synchronize()
    out = dev.cpu().numpy()
    assert np.array_equal(out[:, :k], got[:, :k])
    for s in range(n):
        ref = poisoned[s].copy()
        assert oracle_decode(k, r, ref, er, int(er.sum())) == 0
        assert np.array_equal(out[s], ref)


def test_m16_decode_moves_to_route():
    """A GF(2^16) decode pattern starts on the dense device-built plan and moves to the syndrome route
    once its launches have moved m16_route_min_bytes: the first launch runs k_apply_m16_v1, the second
    k_cs16 + its second stage; both bit-exact vs the oracle."""
    k, r, S, n = 600, 100, 2048, 2
    rng = np.random.default_rng(77)
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    codec = rs_amd.Codec(k, r)
    codec.set_option("m16_route_min_bytes", int(1.5 * n * (k + r) * S))
    codec.encode(dev)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    er = np.zeros(k + r, bool)
    er[rng.choice(k, 80, replace=False)] = True
    er[k + 3] = True
    poisoned = got.copy()
    poisoned[:, er] = 0
    want = poisoned.copy()
    for s in range(n):
        assert oracle_decode(k, r, want[s], er, int(er.sum())) == 0
    kernels = []
    for call in range(3):
        dev.copy_(torch.from_numpy(poisoned))
        codec.decode(dev, er)
        torch.cuda.synchronize()
        kernels.append(codec.last_kernel)
        assert np.array_equal(dev.cpu().numpy(), want), f"call {call} ({codec.last_kernel})"
    assert kernels[0] == "apply_m16_v1" and kernels[1].startswith(CS_DEFAULT + "+") and kernels[2] == kernels[1], kernels


@pytest.mark.parametrize("k,r,t,S", [(1000, 200, 200, 2048), (700, 96, 90, 1024), (4096, 1024, 1024, 1024)])
def test_m16_reenc_decode(k, r, t, S):
    """GF(2^16) decode by re-encoding (information erasures only, t >= 0.9 r): the encode route over the
    surviving information symbols, + the received repair symbols, then the decode matrix's repair
    columns -- bit-exact vs the oracle (C5 shape included), and the same bytes as the plain route."""
    rng = np.random.default_rng(k + r + t)
    n = 2
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    codec = rs_amd.Codec(k, r)
    codec.set_option("m16_route_min_bytes", 0)
    codec.encode(dev)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    er = np.zeros(k + r, bool)
    er[rng.choice(k, t, replace=False)] = True
    poisoned = got.copy()
    poisoned[:, er] = 0
    outs = []
    for reenc in (1, 0):
        codec.set_option("m16_reenc", reenc)
        dev.copy_(torch.from_numpy(poisoned))
        codec.decode(dev, er)
        torch.cuda.synchronize()
        assert codec.last_kernel.startswith(CS_DEFAULT + ("+bs16+xor+" if reenc else "+apply")), codec.last_kernel
        outs.append(dev.cpu().numpy())
    assert np.array_equal(outs[0][:, :k], got[:, :k])
    assert np.array_equal(outs[0], outs[1])
    if k + r <= 1500:
        for s in range(n):
            ref = poisoned[s].copy()
            assert oracle_decode(k, r, ref, er, int(er.sum())) == 0
            assert np.array_equal(outs[0][s], ref)


def test_m16_reenc_when_orbit_stage_is_dense():
    """A re-encode-eligible pattern (information erasures only, t >= 0.9 r) closed under x -> x^16 whose erased
    slots interleave two orbits per coset (slots a, a + 1, a + 4, a + 5, ... of each 16-slot coset): the orbit
    rows do not form runs, so k_bs16 cannot take the plain route's second stage. The route plan is then the
    re-encode decode (rs_route16.cpp:make_plan_route), not the plain route with a dense t x r stage; both
    bit-exact vs the oracle."""
    from _util import oracle_positions
    k, r, S, n = 1000, 256, 1024, 2
    pos = oracle_positions(k, r).astype(np.int64)
    runs, i = [], 0
    while i < k:  # 16-slot cosets among the information slots
        j = i + 1
        while j < k + r and j - i < 16 and pos[j] == (2 * pos[j - 1]) % 65535:
            j += 1
        if j - i == 16 and j <= k:
            runs.append(i)
        i = j
    er = np.zeros(k + r, bool)
    for a in runs[:29]:
        er[[a + d for d in (0, 1, 4, 5, 8, 9, 12, 13)]] = True
    t = int(er.sum())
    assert t == 232 and 10 * t >= 9 * r
    rng = np.random.default_rng(77)
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    codec = rs_amd.Codec(k, r)
    codec.set_option("m16_route_min_bytes", 0)
    codec.encode(dev)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    poisoned = got.copy()
    poisoned[:, er] = 0
    for reenc in (1, 0):
        codec.set_option("m16_reenc", reenc)
        dev.copy_(torch.from_numpy(poisoned))
        codec.decode(dev, er)
        torch.cuda.synchronize()
        if reenc:
            assert "+bs16+xor+" in codec.last_kernel, codec.last_kernel
        else:
            assert codec.last_kernel.startswith(CS_DEFAULT + "+apply"), codec.last_kernel
        out = dev.cpu().numpy()
        for s in range(n):
            ref = poisoned[s].copy()
            assert oracle_decode(k, r, ref, er, t) == 0
            assert np.array_equal(out[s], ref), (reenc, s)


def test_drop_in_arena_mixed_layouts():
    """Per-call calls on seq_create memory in layouts other than one strided sequence: information and
    repair symbols in two different sequences (zero-copy with two bases), and a sequence whose symbol
    pointers were permuted (no longer one strided run: the gather / scatter path for that side) --
    bit-exact vs the oracle."""
    k, r, S = 128, 32, 65536
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    want = np.zeros((k + r, S), np.uint8)
    want[:k] = data
    assert oracle_encode(k, r, want) == 0
    rs = rs_amd.RS()
    qa, qb = rs_amd.Seq(k, S), rs_amd.Seq(r, S)
    for i in range(k):
        qa.symbols[i][:] = data[i]
    for call in range(3):  # first call: DMA; then the specialised XOR kernel zero-copy
        va, vb = qa.view(0, k), qb.view(0, r)
        assert rs_amd._lib.rs_generate_repair_symbols(rs._h, ctypes.byref(va), ctypes.byref(vb)) == 0
        assert np.array_equal(np.stack(qb.symbols), want[k:]), f"two sequences, call {call}"
    qa.close()
    qb.close()
    q = rs_amd.Seq(k + r, S)
    for i in range(k):
        q.symbols[i][:] = data[i]
    ptrs = q._p.contents.symbols
    sym_p = ctypes.POINTER(rs_amd.SymbolT)
    a0, a1 = (ctypes.cast(ptrs[i], ctypes.c_void_p).value for i in (0, 1))  # addresses, not views of the slots
    ptrs[0], ptrs[1] = ctypes.cast(a1, sym_p), ctypes.cast(a0, sym_p)  # logical symbol 0 = second block row
    ref = np.zeros_like(want)
    ref[:k] = want[:k]
    ref[[0, 1]] = ref[[1, 0]]
    assert oracle_encode(k, r, ref) == 0
    er = rs_amd.bench_pattern(k, r)
    for call in range(4):
        assert rs.generate_repair_symbols(q, r) == 0
        got = np.stack([np.ctypeslib.as_array(ptrs[i].contents.data, (S,)) for i in range(k + r)])
        assert np.array_equal(got, ref), f"permuted, encode call {call}"
        for i in np.nonzero(er)[0]:
            np.ctypeslib.as_array(ptrs[i].contents.data, (S,))[:] = 0
        assert rs.restore_symbols(k, r, q, er, int(er.sum())) == 0
        got = np.stack([np.ctypeslib.as_array(ptrs[i].contents.data, (S,)) for i in range(k + r)])
        assert np.array_equal(got[:k], ref[:k]), f"permuted, restore call {call}"
    ptrs[0], ptrs[1] = ctypes.cast(a0, sym_p), ctypes.cast(a1, sym_p)
    q.close()
    rs.close()


def test_drop_in_m16_large_symbols():
    """Reference per-call API on a GF(2^16) code with 64 KiB symbols: the call is pipelined in column
    chunks on one stream and each chunk's small grid runs split-K; encode + restore bit-exact vs the
    oracle, twice (second call reuses the plans and the split-K scratch)."""
    k, r, S = 300, 64, 65536
    rng = np.random.default_rng(64)
    rs = rs_amd.RS()
    for rep in range(2):
        syms = [np.zeros(S, np.uint8) for _ in range(k + r)]
        for i in range(k):
            syms[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
        assert rs.generate_repair_symbols(syms[:k], syms[k:]) == 0
        want = np.stack(syms).copy()
        ref = want.copy()
        ref[k:] = 0
        assert oracle_encode(k, r, ref) == 0
        assert np.array_equal(want, ref)
        er = np.zeros(k + r, bool)
        er[rng.choice(k + r, r, replace=False)] = True
        for i in np.nonzero(er)[0]:
            syms[i][:] = 0
        assert rs.restore_symbols(k, r, syms, er, int(er.sum())) == 0
        got = np.stack(syms)
        assert np.array_equal(got[:k], want[:k]), f"call {rep}"
    rs.close()


@pytest.mark.parametrize("k,r,S,pattern", [(128, 32, 65536, "bench"), (128, 32, 65536, "span"),
                                           (128, 32, 65536, "random"), (300, 64, 8192 + 6, "random"),
                                           (64, 16, 16384 + 2, "bench"), (4, 2, 256, "random"),
                                           (10, 4, 4096, "bench"), (200, 55, 66, "random"),
                                           (300, 64, 64, "random"), (300, 70, 1024, "random"),
                                           (300, 64, 16384, "random"), (128, 32, 32768, "span")])
def test_drop_in_pinned_seq(k, r, S, pattern):
    """seq_create places sequences in page-locked memory (own block from 1 MiB, slab share below) and
    the per-call API works on them in place: zero-copy launches (specialised XOR kernels; any kernel on
    stripes up to 1 MiB), else 2D DMA in and restored rows out by DMA of their span or k_put_rows.
    Encode and restore bit-exact vs the oracle for scattered (bench, random) and contiguous (span)
    erasures, GF(16) / GF(256) / GF(2^16) codes, symbol sizes that are not multiples of 16 (padded
    pitch); the same calls on separately allocated symbols (RS_AMD_PINNED_SEQ=0 -> symbol_create per
    symbol: from 16 KiB page-aligned buffers page-locked at creation, moved by gather / scatter kernels
    when S is a multiple of 16; else calloc and host copies) give the same bytes."""
    import os
    rng = np.random.default_rng(k * 7 + S)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    if pattern == "bench":
        er = rs_amd.bench_pattern(k, r)
    elif pattern == "span":
        er = np.zeros(k + r, bool)
        er[5:5 + r] = True
    else:
        er = np.zeros(k + r, bool)
        er[rng.choice(k + r, r, replace=False)] = True
    want = np.zeros((k + r, S), np.uint8)
    want[:k] = data
    assert oracle_encode(k, r, want) == 0
    rs = rs_amd.RS()
    outs = []
    for flag in ("1", "0"):
        os.environ["RS_AMD_PINNED_SEQ"] = flag
        try:
            q = rs_amd.Seq(k + r, S)
        finally:
            os.environ.pop("RS_AMD_PINNED_SEQ")
        pitch = q.symbols[1].ctypes.data - q.symbols[0].ctypes.data
        if flag == "1":
            assert pitch == _pad(S), "seq_create did not place the sequence in one arena"
        for i in range(k):
            q.symbols[i][:] = data[i]
        # symbol_create buffers from 16 KiB: page-aligned, registered on first use (a block taken back from
        # the idle pool keeps its registration)
        own = S >= 16384 and flag == "0"
        assert all(rs_amd.symbol_registered(x) in ((0, 1) if own else (-1,)) for x in q.symbols)
        for call in range(4):  # decode calls 3+ of a GF(256) pattern run the specialised plan, 4+ zero-copy
            assert rs.generate_repair_symbols(q, r) == 0
            # registered by the call when the registered-symbol path takes them (S a multiple of 16)
            assert all(rs_amd.symbol_registered(x) == ((1 if S % 16 == 0 else 0) if own else -1) for x in q.symbols)
            got = np.stack(q.symbols)
            assert np.array_equal(got, want), f"encode pinned={flag} call {call}"
            for i in np.nonzero(er)[0]:
                q.symbols[i][:] = 0
            assert rs.restore_symbols(k, r, q, er, int(er.sum())) == 0
            got = np.stack(q.symbols)
            assert np.array_equal(got[:k], data), f"restore pinned={flag} call {call}"
            assert not got[k:][er[k:]].any()  # erased repair slots are not written
        outs.append(got)
        q.close()
    assert np.array_equal(outs[0], outs[1])
    rs.close()



def test_registered_symbol_retired_past_pool_cap():
    """The round-3 fault's mechanism, checked once ("registered caller symbols"):
    symbol_create pages registered by a per-call use and destroyed past the idle pool's cap are
    unregistered with the result checked (unregistrations + n, no failure, no stuck block), their memory
    is returned (the pages are PROT_NONE) while the address range stays reserved, later symbols never get
    those addresses, and a torch D2H copy into fresh pageable memory afterwards is exact."""
    k, r, S = 10, 4, 65536
    n = k + r
    rng = np.random.default_rng(404)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    want = np.zeros((n, S), np.uint8)
    want[:k] = data
    assert oracle_encode(k, r, want) == 0
    old_cap = rs_amd.symbol_pool_cap(0)  # nothing parks: every destroyed block is unregistered and retired
    try:
        st0 = rs_amd.symbol_stats()
        os.environ["RS_AMD_PINNED_SEQ"] = "0"
        try:
            q = rs_amd.Seq(n, S)
        finally:
            os.environ.pop("RS_AMD_PINNED_SEQ")
        assert all(rs_amd.symbol_registered(x) == 0 for x in q.symbols)  # symbol_create made no HIP call
        for i in range(k):
            q.symbols[i][:] = data[i]
        rs = rs_amd.RS()
        assert rs.generate_repair_symbols(q, r) == 0
        assert np.array_equal(np.stack(q.symbols), want)
        assert all(rs_amd.symbol_registered(x) == 1 for x in q.symbols)
        addrs = [x.ctypes.data for x in q.symbols]
        q.close()
        rs.close()
        st1 = rs_amd.symbol_stats()
        assert st1["registrations"] - st0["registrations"] == n
        assert st1["unregistrations"] - st0["unregistrations"] == n
        assert st1["unregister_failures"] == st0["unregister_failures"]
        assert st1["stuck_blocks"] == st0["stuck_blocks"]
        assert st1["retired_blocks"] - st0["retired_blocks"] == n
        assert st1["pinned_bytes"] == st0["pinned_bytes"]
        with open("/proc/self/maps") as f:
            maps = [(int(a, 16), int(b, 16), perms) for a, b, perms in
                    ((ln.split()[0].split("-") + [ln.split()[1]]) for ln in f)]
        for a in addrs:
            assert any(lo <= a < hi and perms == "---p" for lo, hi, perms in maps), "retired pages still mapped"
        os.environ["RS_AMD_PINNED_SEQ"] = "0"
        try:
            q2 = rs_amd.Seq(n, S)
        finally:
            os.environ.pop("RS_AMD_PINNED_SEQ")
        assert not set(x.ctypes.data for x in q2.symbols) & set(addrs)
        q2.close()
        src = torch.randint(0, 256, (8, 1 << 20), dtype=torch.uint8, device="cuda")
        ref = src.sum(dim=1, dtype=torch.int64).cpu()
        for _ in range(3):
            host = src.cpu()  # pageable destination
            assert torch.equal(host.sum(dim=1, dtype=torch.int64), ref)
    finally:
        rs_amd.symbol_pool_cap(old_cap)


@pytest.mark.parametrize("k,r,S,n,pinned", [(128, 32, 65536, 30, True), (10, 4, 4096 + 24, 300, False),
                                            (300, 70, 2048 + 10, 5, True)])
def test_host_memory_batches(k, r, S, n, pinned):
    """rsg_encode_host / rsg_decode_host on stripes in host memory (pinned and pageable; C3 shape in
    two device batches; GF(2^16) code; tail columns): bit-exact vs the oracle."""
    rng = np.random.default_rng(k + r + n)
    host = torch.zeros((n, k + r, S), dtype=torch.uint8)
    if pinned:
        host = host.pin_memory()
    host[:, :k] = torch.from_numpy(rng.integers(0, 256, (n, k, S), dtype=np.uint8))
    codec = rs_amd.Codec(k, r)
    codec.encode_host(host)
    got = host.numpy().copy()
    for s in range(0, n, max(1, n // 4)):
        want = got[s].copy()
        want[k:] = 0
        assert oracle_encode(k, r, want) == 0
        assert np.array_equal(got[s], want), f"encode stripe {s}"
    er = np.zeros(k + r, bool)
    er[1 + rng.choice(k + r - 1, r - 1, replace=False)] = True
    er[0] = True  # r erasures, information slot 0 among them
    host[:, torch.from_numpy(er)] = 0
    codec.decode_host(host, er)
    out = host.numpy()
    assert np.array_equal(out[:, :k], got[:, :k])
    assert not out[:, k:][:, er[k:]].any()  # erased repair slots are not written


def test_release_build_ignores_diagnostic_knobs():
    """The product library rejects the ablation options (RS_ERR_INVALID) and ignores every RS_XJ_*
    environment variable when it generates the kernels it launches: with ablation and generation knobs
    set, a fresh process still encodes and decodes bit-exactly through the same XOR kernel (same content
    hash in its name) as without them."""
    codec = rs_amd.Codec(128, 32)
    # ablations / stamps, and (round 5) the option-only A/B families, overlap variants and block layouts
    for name, value in ([("m8_mode", v) for v in (0, 1, 2, 3, 4, 10, 11, 12, 13, 14, 15, 16, 17, 19, 21)]
                        + [("m16_mode", 1), ("stamp_buffer", 1), ("m16_cs_col", 1024), ("m16_cs_overlap", 1),
                           ("m8_syn_overlap", 1), ("m8_ps_cpb", 2), ("m8_syn_coord", 1)]
                        + [("m8_ps_kernel", v) for v in (1, 2, 4, 5, 6, 7, 8, 9, 11)]):
        with pytest.raises(rs_amd.RSError):
            codec.set_option(name, value)
    for name, value in [("m8_mode", 18), ("m8_mode", 20), ("m8_ps_kernel", 0), ("m8_ps_kernel", 3),
                        ("m8_ps_kernel", 10), ("m16_cs_col", 256),
                        ("m16_cs_overlap", 0), ("m8_syn_overlap", 0), ("m8_ps_cpb", 1), ("xj", 0), ("xj", 1)]:
        codec.set_option(name, value)  # the production settings stay accepted
    import os
    import subprocess
    import sys
    code = r"""
import numpy as np, torch, rs_amd, sys
sys.path.insert(0, sys.argv[1])
from _util import gen_info, oracle_encode, oracle_decode
k, r, S, n = 128, 32, 4096, 3
host = np.zeros((n, k + r, S), np.uint8)
for s in range(n): host[s, :k] = gen_info(7, s, k * S).reshape(k, S)
dev = torch.from_numpy(host).cuda()
c = rs_amd.Codec(k, r)
c.encode(dev); torch.cuda.synchronize()
assert c.last_kernel.startswith("rs_xj"), c.last_kernel
got = dev.cpu().numpy()
for s in range(n):
    want = host[s].copy(); assert oracle_encode(k, r, want) == 0
    assert np.array_equal(got[s], want), s
er = rs_amd.bench_pattern(k, r)
for _ in range(2):
    dev[:, torch.from_numpy(er)] = 0xA5
    c.decode(dev, er); torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy()[:, :k], got[:, :k])
print("ok", c.last_kernel)
"""
    here = os.path.dirname(os.path.abspath(__file__))
    base = dict(os.environ, PYTHONPATH=os.path.dirname(rs_amd.__file__))
    for k in [v for v in base if v.startswith("RS_XJ_")]:
        base.pop(k)
    plain = subprocess.run([sys.executable, "-c", code, here], env=base, capture_output=True, text=True, timeout=300)
    assert plain.returncode == 0 and plain.stdout.startswith("ok rs_xj"), plain.stdout + plain.stderr
    # neither the ablations nor the generation knobs change the shipped kernel (same content hash)
    env = dict(base, RS_XJ_ABLATE="1", RS_XJ_ALIAS="1", RS_XJ_OPR="8", RS_XJ_EARLY="0", RS_XJ_HORNER="1")
    p = subprocess.run([sys.executable, "-c", code, here], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and p.stdout.startswith("ok rs_xj"), p.stdout + p.stderr
    assert p.stdout.split()[-1] == plain.stdout.split()[-1], (p.stdout, plain.stdout)


@pytest.mark.parametrize("name", EXTRA_CASES)
def test_golden_symbol_ops_and_transforms(name):
    """gf_add / gf_mul / gf_madd and fft_transform(_cycl) / fft_partial_transform(_cycl) through the C ABI
    (host symbols in, GPU compute, host symbols out) against the reference's outputs."""
    c = case(name)
    S = c["S"]
    if c["op"].startswith("gf_"):
        a, b = extra_inputs(c)
        a = a.copy()
        gf = rs_amd.lib.gf_create()
        {"gf_add": lambda: rs_amd.symbol_add(a, b), "gf_mul": lambda: rs_amd.symbol_mul(a, c["t"], gf),
         "gf_madd": lambda: rs_amd.symbol_madd(a, c["t"], b, gf)}[c["op"]]()
        rs_amd.lib.gf_destroy(gf)
        check_golden(c, a.tobytes())
        return
    f, arg = extra_inputs(c)
    res = [np.full(S, 0xA5, np.uint8) for _ in range(c["r"])]  # outputs are overwritten
    kind = {"fft_t": "transform", "fft_tc": "transform_cycl", "fft_p": "partial", "fft_pc": "partial_cycl"}[c["op"]]
    gf = rs_amd.lib.gf_create()
    rc = rs_amd.fft(kind, [np.ascontiguousarray(x) for x in f], res, arg, gf)
    rs_amd.lib.gf_destroy(gf)
    assert rc == c["rc"]
    check_golden(c, b"".join(x.tobytes() for x in res))


def test_symbol_ops_large_and_aliased():
    """gf_madd over a 1 MiB symbol and gf_add with a == b (zeroes it), vs the numpy restatement."""
    from _util import gf_tables
    exp, log = gf_tables()
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    b = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    wa, wb = a.view("<u2").astype(np.int64), b.view("<u2").astype(np.int64)
    want = wa ^ np.where(wb != 0, exp[(log[wb] + log[40000]) % 65535], 0)
    rs_amd.symbol_madd(a, 40000, b)
    assert np.array_equal(a.view("<u2"), want.astype(np.uint16))
    rs_amd.symbol_add(a, a)
    assert not a.any()


def test_reference_surface_program(tmp_path):
    """tests/c/ref_surface.c calls every function of the reference's rs/ and memory/ headers, built
    against this repo's headers and linked against librs_amd.so, including the call patterns of the
    reference's src/example.c and test_random_data.c (100 self-checked rounds); its outputs equal the
    goldens (ex_*, c1_*, c3_* and the secondary-surface cases)."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "ref_surface")
    assert os.path.exists(exe), "build it with make -C tests/c (part of __graft_entry__.build)"
    p = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    for name in ("gf_add_64", "gf_mul_c", "gf_madd_c", "fft_t_small", "fft_tc_small", "fft_p_small", "fft_pc_mixed",
                 "c1_enc", "c1_dec_info_rep", "ex_enc", "ex_dec", "c3_enc", "c3_dec_bench", "c3_dec_rand17",
                 "odd_enc_9", "odd_dec_9", "odd_enc_4097", "odd_dec_4097"):
        check_golden(case(name), (tmp_path / f"{name}.bin").read_bytes())


@pytest.mark.parametrize("lost", ["scattered", "contiguous"])
def test_drop_in_m8_repeated_pattern_chunked(lost):
    """Per-call restore of one pattern, 5 calls on a GF(256) code with 64 KiB symbols: the first two run
    the generic kernel over the whole symbol, the third specialises the plan and from then on the call is
    pipelined in 4 column chunks. Every call bit-exact vs the oracle, for a scattered lost set (rows
    packed on the device, k_gather_rows) and a contiguous one (one span copied back)."""
    k, r, S = 128, 32, 65536
    rng = np.random.default_rng(81 if lost == "scattered" else 82)
    er = np.zeros(k + r, bool)
    if lost == "scattered":
        er[rng.choice(k, 20, replace=False)] = True
        er[k + rng.choice(r, 5, replace=False)] = True
    else:
        er[40:64] = True
    rs = rs_amd.RS()
    for call in range(5):
        syms = [np.zeros(S, np.uint8) for _ in range(k + r)]
        for i in range(k):
            syms[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
        assert rs.generate_repair_symbols(syms[:k], syms[k:]) == 0
        full = np.stack(syms).copy()
        for i in np.nonzero(er)[0]:
            syms[i][:] = 0
        ref = np.stack(syms).copy()
        assert rs.restore_symbols(k, r, syms, er, int(er.sum())) == 0
        assert oracle_decode(k, r, ref, er, int(er.sum())) == 0
        got = np.stack(syms)
        assert np.array_equal(got, ref), f"call {call}"
        assert np.array_equal(got[:k], full[:k]), f"call {call}"
    rs.close()


def test_new_pattern_does_not_stall_other_streams():
    """A decode with a new erasure pattern builds its plan on the caller's stream (pinned upload, no
    null-stream copy): while another (blocking) stream is busy with a long encode, the decode call
    returns with that stream still running, and its result is bit-exact."""
    if rs_amd._lib.rsg_check_enabled():
        pytest.skip("RS_AMD_CHECK: every launch waits for the device by design")
    hip = ctypes.CDLL("libamdhip64.so")
    k, r, S = 128, 32, 65536
    busy = torch.empty((1024, k + r, S), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(busy, k, 3)
    small = torch.zeros((4, k + r, 4096), dtype=torch.uint8, device="cuda")
    rs_amd.fill_info(small, k, 4)
    codec = rs_amd.Codec(k, r)
    codec.encode(small)
    codec.encode(busy[:1])  # encode kernel loaded
    torch.cuda.synchronize()
    full = small.cpu().numpy()
    sa, sb = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(sa)) == 0  # default flags: a blocking stream
    assert hip.hipStreamCreateWithFlags(ctypes.byref(sb), 1) == 0
    rng = np.random.default_rng(11)
    try:
        for trial in range(3):
            er = np.zeros(k + r, bool)
            er[rng.choice(k + r, 25, replace=False)] = True
            er[trial] = True  # a new pattern with at least one information erasure
            small.copy_(torch.from_numpy(full))  # the last trial left its erased repair slots zero
            small[:, torch.from_numpy(er)] = 0
            torch.cuda.synchronize()
            for _ in range(30):  # ~90 ms of encode work on the blocking stream
                assert codec.encode(busy, stream=sa.value) == 0
            assert codec.decode(small, er, stream=sb.value) == 0
            still_busy = hip.hipStreamQuery(sa) != 0  # hipErrorNotReady
            assert hip.hipStreamSynchronize(sb) == 0 and hip.hipStreamSynchronize(sa) == 0
            assert still_busy, "the decode call waited for the other stream"
            assert np.array_equal(small.cpu().numpy()[:, :k], full[:, :k]), trial
    finally:
        hip.hipStreamDestroy(sa)
        hip.hipStreamDestroy(sb)


@pytest.mark.parametrize("k,r", [(4, 2), (128, 32), (300, 60)])
def test_edge_empty_batches_and_no_erasures(k, r):
    """Edge cases of the batched API: zero stripes (encode / decode return 0 and touch nothing), a decode
    with no erasure (t = 0: nothing to restore, the stripes stay bit-identical), and a pattern that loses
    only repair symbols (the reference restores information symbols only, so nothing changes either)."""
    S = 2048
    rng = np.random.default_rng(k + r)
    host = np.zeros((3, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (3, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    codec = rs_amd.Codec(k, r)
    assert codec.encode(dev[:0]) == 0
    codec.encode(dev)
    torch.cuda.synchronize()
    enc = dev.cpu().numpy()
    want = host.copy()
    for s in range(3):
        assert oracle_encode(k, r, want[s]) == 0
    assert np.array_equal(enc, want)
    none = np.zeros(k + r, bool)
    assert codec.decode(dev, none) == 0
    rep_only = none.copy()
    rep_only[k + rng.choice(r, min(r, 2), replace=False)] = True
    poisoned = enc.copy()
    poisoned[:, rep_only] = 0
    dev.copy_(torch.from_numpy(poisoned))
    assert codec.decode(dev, rep_only) == 0
    er = none.copy()
    er[:min(k, r)] = True
    assert codec.decode(dev[:0], er) == 0
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), poisoned)


# ------------------------------------------------------------------ batched symbol ops (rsg_symbol_ops)
def _ops_numpy(mem, ops, S):
    """Sequential restatement of a batch (reference gf65536.c:155-219 per op): mem maps address -> uint8 array."""
    from _util import gf_tables
    exp, log = gf_tables()
    nw = S // 2

    def mul(c, w):
        return np.where(w != 0, exp[(log[w] + log[c]) % 65535], 0) if c else np.zeros_like(w)
    for op, a, b, c in ops:
        wa = mem[a][:2 * nw].view("<u2").astype(np.int64)
        if op == rs_amd.OP_MUL:
            wa = mul(c, wa)
        else:
            wb = mem[b][:2 * nw].view("<u2").astype(np.int64)
            wa = wa ^ (wb if op == rs_amd.OP_ADD else mul(c, wb))
        mem[a][:2 * nw] = wa.astype("<u2").view(np.uint8)


def test_symbol_ops_batch_vs_goldens():
    """Every gf_add / gf_mul / gf_madd golden of the reference (coefficients 0, 1 and general; odd symbol
    sizes leave the last byte untouched) through ONE rsg_symbol_ops batch per symbol size, on device memory."""
    from _util import extra_inputs
    by_size = {}
    for name in EXTRA_CASES:
        c = case(name)
        if c["op"].startswith("gf_"):
            by_size.setdefault(c["S"], []).append(c)
    for S, cases in by_size.items():
        P = (S + 15) // 16 * 16
        dev = torch.zeros((2 * len(cases), P), dtype=torch.uint8, device="cuda")
        ops = []
        for i, c in enumerate(cases):
            a, b = extra_inputs(c)
            dev[2 * i, :S] = torch.from_numpy(a)
            dev[2 * i + 1, :S] = torch.from_numpy(b)
            kind = {"gf_add": rs_amd.OP_ADD, "gf_mul": rs_amd.OP_MUL, "gf_madd": rs_amd.OP_MADD}[c["op"]]
            ops.append((kind, dev[2 * i].data_ptr(), dev[2 * i + 1].data_ptr(), c["t"]))
        rs_amd.symbol_ops(ops, S)
        torch.cuda.synchronize()
        out = dev.cpu().numpy()
        for i, c in enumerate(cases):
            check_golden(c, out[2 * i, :S].tobytes())


@pytest.mark.parametrize("S", [4096, 4096 + 2, 1024 + 6, 65536, 9])
def test_symbol_ops_chains_vs_numpy(S):
    """Random batches shaped like the reference's loops over gf_* (_rs_get_evaluator_poly, _rs_restore_erased:
    many madds accumulating into few targets), with gf_mul / gf_add in the chains, sources equal to their own
    target, coefficients 0 and 1, targets and sources interleaved in one buffer: bit-exact against the ops
    applied one after another on the CPU."""
    rng = np.random.default_rng(S)
    n_t, n_s, n_ops = 24, 40, 600
    P = (S + 15) // 16 * 16
    host = rng.integers(0, 256, (n_t + n_s, P), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    addr = [dev[i].data_ptr() for i in range(n_t + n_s)]
    ops = []
    for _ in range(n_ops):
        t = int(rng.integers(n_t))
        kind = int(rng.choice([rs_amd.OP_ADD, rs_amd.OP_MUL, rs_amd.OP_MADD], p=[0.15, 0.1, 0.75]))
        src = t if rng.random() < 0.05 else n_t + int(rng.integers(n_s))
        coef = int(rng.choice([0, 1, int(rng.integers(2, 65536))], p=[0.05, 0.05, 0.9]))
        ops.append((kind, addr[t], addr[src], coef))
    rs_amd.symbol_ops(ops, S)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    mem = {addr[i]: host[i].copy() for i in range(n_t + n_s)}
    _ops_numpy(mem, ops, S)
    want = np.stack([mem[addr[i]] for i in range(n_t + n_s)])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("S,lens", [(1024 + 6, [1, 3, 7, 64, 100, 203]), (65536, [150, 149, 37, 5]),
                                    (9, [40, 2, 77]), (4096, [8, 9, 31, 33, 64, 65])])
def test_symbol_ops_split_chains_vs_numpy(S, lens):
    """Few long chains (gf_madd / gf_add, coefficients 0 / 1 / general) make the library cut each chain into
    slices on several waves of one workgroup (rs_symops.hip) and XOR the slice results; the two chains with a
    gf_mul or a self-source op in the middle (the target scaled) multiply each slice's result by the later
    slices' scale factors first (kChainAffine). Bit-exact against the ops applied one after another."""
    rng = np.random.default_rng(len(lens) * 1000 + S)
    n_s = 48
    n_t = len(lens) + 2
    P = (S + 15) // 16 * 16
    host = rng.integers(0, 256, (n_t + n_s, P), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    addr = [dev[i].data_ptr() for i in range(n_t + n_s)]
    per_target = []
    for t, n in enumerate(lens + [30, 30]):
        ops = []
        for i in range(n):
            kind = int(rng.choice([rs_amd.OP_ADD, rs_amd.OP_MADD], p=[0.2, 0.8]))
            coef = int(rng.choice([0, 1, int(rng.integers(2, 65536))], p=[0.05, 0.05, 0.9]))
            ops.append((kind, addr[t], addr[n_t + int(rng.integers(n_s))], coef))
        if t == len(lens):  # not a pure sum: a scale in the middle
            ops[15] = (rs_amd.OP_MUL, addr[t], 0, int(rng.integers(2, 65536)))
        if t == len(lens) + 1:  # a self-source madd: (1 + c) a
            ops[10] = (rs_amd.OP_MADD, addr[t], addr[t], int(rng.integers(2, 65536)))
        per_target.append(ops)
    ops = [o for i in range(max(map(len, per_target))) for tl in per_target if i < len(tl) for o in [tl[i]]]
    rs_amd.symbol_ops(ops, S)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    mem = {addr[i]: host[i].copy() for i in range(n_t + n_s)}
    _ops_numpy(mem, ops, S)
    want = np.stack([mem[addr[i]] for i in range(n_t + n_s)])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("S", [1024 + 6, 4096, 9])
def test_symbol_ops_split_scaling_chains(S):
    """Split chains that scale their target at chosen places: a gf_mul first and last, gf_mul by 0 and by 1,
    a self gf_add (zeroes the target) and self gf_madds ((1 + c) a, incl. c = 1) at slice starts, ends and
    middles, chains of every length 1 .. 64 so every slice count and ragged last slice occurs. Each slice's result
    times the later slices' scale factors, XORed: bit-exact against the ops applied one after another."""
    rng = np.random.default_rng(S + 5)
    n_s = 16
    lens = list(range(1, 65, 3))
    n_t = len(lens)
    P = (S + 15) // 16 * 16
    host = rng.integers(0, 256, (n_t + n_s, P), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    addr = [dev[i].data_ptr() for i in range(n_t + n_s)]
    special = [lambda t: (rs_amd.OP_MUL, addr[t], 0, int(rng.integers(2, 65536))),
               lambda t: (rs_amd.OP_MUL, addr[t], 0, 0), lambda t: (rs_amd.OP_MUL, addr[t], 0, 1),
               lambda t: (rs_amd.OP_ADD, addr[t], addr[t], 0),
               lambda t: (rs_amd.OP_MADD, addr[t], addr[t], int(rng.integers(2, 65536))),
               lambda t: (rs_amd.OP_MADD, addr[t], addr[t], 1)]
    per_target = []
    for t, n in enumerate(lens):
        ops = [(rs_amd.OP_MADD, addr[t], addr[n_t + int(rng.integers(n_s))], int(rng.integers(1, 65536)))
               for _ in range(n)]
        for pos in {0, n - 1, n // 2, n // 3, (2 * n) // 3}:
            if rng.random() < 0.8:
                ops[pos] = special[int(rng.integers(len(special)))](t)
        per_target.append(ops)
    ops = [o for i in range(max(lens)) for tl in per_target if i < len(tl) for o in [tl[i]]]
    rs_amd.symbol_ops(ops, S)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    mem = {addr[i]: host[i].copy() for i in range(n_t + n_s)}
    _ops_numpy(mem, ops, S)
    want = np.stack([mem[addr[i]] for i in range(n_t + n_s)])
    assert np.array_equal(got, want)


def test_symbol_ops_more_chains_than_one_launch():
    """More targets than one launch's grid takes (65535 chains per launch): the chain launches share one
    op array and one constants array (k_symop_consts runs once per call over every op), so the later
    launches' chains index ops and constants past the first launch's. Bit-exact against numpy."""
    from _util import gf_tables
    exp, log = gf_tables()
    S, n_t, n_s = 16, 70001, 8
    rng = np.random.default_rng(70001)
    tgt = torch.from_numpy(rng.integers(0, 256, (n_t, S), dtype=np.uint8)).cuda()
    src = torch.from_numpy(rng.integers(0, 256, (n_s, S), dtype=np.uint8)).cuda()
    t0 = tgt.cpu().numpy().view("<u2").astype(np.int64)
    ws = src.cpu().numpy().view("<u2").astype(np.int64)
    j1, j2 = rng.integers(0, n_s, n_t), rng.integers(0, n_s, n_t)
    c1, c2 = rng.integers(2, 65536, n_t), rng.integers(0, 65536, n_t)
    ops = np.zeros(2 * n_t, rs_amd.SYMBOL_OP_DTYPE)
    ops["a"] = tgt.data_ptr() + np.repeat(np.arange(n_t, dtype=np.uint64), 2) * S
    ops["op"] = np.tile([rs_amd.OP_MADD, rs_amd.OP_MUL], n_t)
    ops["b"][0::2] = src.data_ptr() + j1.astype(np.uint64) * S
    ops["b"][1::2] = src.data_ptr() + j2.astype(np.uint64) * S  # ignored by gf_mul
    ops["coef"][0::2], ops["coef"][1::2] = c1, c2
    rs_amd.symbol_ops(ops, S)
    torch.cuda.synchronize()

    def mul(c, w):  # c per row, w [n, words]
        lw = np.where(w != 0, log[w], -1)
        out = np.where((lw >= 0) & (c[:, None] != 0), exp[(lw + log[c][:, None]) % 65535], 0)
        return out
    want = mul(c2, t0 ^ mul(c1, ws[j1]))
    assert np.array_equal(tgt.cpu().numpy().view("<u2").astype(np.int64), want)


def test_symbol_ops_back_to_back_calls_and_streams():
    """More calls than staging slots, on two streams, before any synchronisation (each call's op list must
    survive until its kernel read it), then a reference-style evaluator loop Omega = S * Lambda mod x^r as one
    batch on the result."""
    S, n = 2048, 12
    rng = np.random.default_rng(3)
    host = rng.integers(0, 256, (2 * n, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    mem = {dev[i].data_ptr(): host[i].copy() for i in range(2 * n)}
    all_ops = []
    for call in range(10):
        i = call % n
        ops = [(rs_amd.OP_MADD, dev[i].data_ptr(), dev[n + j].data_ptr(), int(rng.integers(1, 65536)))
               for j in range(n)]
        st = streams[call % 2]
        st.wait_stream(streams[(call + 1) % 2])  # calls on one target are ordered by the caller
        rs_amd.symbol_ops(ops, S, stream=st)
        all_ops += ops
    torch.cuda.synchronize()
    _ops_numpy(mem, all_ops, S)
    assert np.array_equal(dev.cpu().numpy(), np.stack([mem[dev[i].data_ptr()] for i in range(2 * n)]))
    # evaluator: om[i + j] ^= lam[i] * syn[j] (reference reed_solomon.c:235-245), targets om, sources syn
    r = 8
    syn = torch.from_numpy(rng.integers(0, 256, (r, S), dtype=np.uint8)).cuda()
    om = torch.zeros((r, S), dtype=torch.uint8, device="cuda")
    lam = [int(x) for x in rng.integers(0, 65536, r)]
    ops = [(rs_amd.OP_MADD, om[i + j].data_ptr(), syn[j].data_ptr(), lam[i]) for i in range(r) for j in range(r - i)]
    rs_amd.symbol_ops(ops, S)
    torch.cuda.synchronize()
    m2 = {om[i].data_ptr(): np.zeros(S, np.uint8) for i in range(r)}
    m2.update({syn[j].data_ptr(): syn[j].cpu().numpy() for j in range(r)})
    _ops_numpy(m2, ops, S)
    assert np.array_equal(om.cpu().numpy(), np.stack([m2[om[i].data_ptr()] for i in range(r)]))
