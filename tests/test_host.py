"""CPU tests of the product library's host side: the C ABI loads and exports every declared entry
point, the coding matrices equal the reference's linear maps (golden fixtures), the GF(256)^2
coordinate arithmetic of the m <= 8 kernels is exact, and the hiprtc specialiser compiles.
No GPU compute is called here."""
import hashlib
import os
import re

import numpy as np
import pytest

import rs_amd
from _util import EXTRA_OPS, REPO, case, case_inputs, check_golden, gf_apply, gf_tables, manifest, run_case_oracle

HEADERS = ["include/rs/reed_solomon.h", "include/rs/gf65536.h", "include/rs/cyclotomic_coset.h", "include/rs/fft.h",
           "include/memory/seq.h", "include/memory/symbol.h", "include/rs_amd/rsg.h"]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(os.path.join(REPO, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\([^;{]*\)\s*;", src, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 30, names
    missing = [n for n in names if not hasattr(rs_amd.lib, n)]
    assert not missing, missing


def test_scalar_kats_through_library():
    L = rs_amd.lib
    gf = L.gf_create()
    try:
        assert L.gf_mul_ee(gf, 31981, 38739) == 42167
        assert L.gf_mul_ee(gf, 58263, 29917) == 33120
        assert L.gf_div_ee(gf, 12320, 29623) == 11439
        assert L.gf_div_ee(gf, 5768, 15888) == 24163
        assert L.gf_get_normal_basis_element(gf, 8, 0) == 16402
    finally:
        L.gf_destroy(gf)
    assert L.cc_get_coset_size(21845) == 2 and L.cc_get_coset_size(257) == 8 and L.cc_get_coset_size(1) == 16


def _select(k, r):
    L = rs_amd.lib
    ci, cr = np.zeros(1, np.uint16), np.zeros(1, np.uint16)
    L.cc_estimate_cosets_cnt(k, r, ci.ctypes.data, cr.ctypes.data)
    inf = np.zeros(int(ci[0]) * 2, np.uint16)  # coset_t = {u16 leader, u8 size} padded to 4 bytes
    rep = np.zeros(int(cr[0]) * 2, np.uint16)
    ni, nr = np.zeros(1, np.uint16), np.zeros(1, np.uint16)
    cc = L.cc_create()
    L.cc_select_cosets(cc, k, r, inf.ctypes.data, int(ci[0]), ni.ctypes.data, rep.ctypes.data, int(cr[0]),
                       nr.ctypes.data)
    L.cc_destroy(cc)
    f = lambda a, n: [(int(a[2 * i]), int(a[2 * i + 1] & 0xFF)) for i in range(int(n[0]))]
    return f(inf, ni), f(rep, nr)


def test_cc_select_cosets_kat_through_library():
    # test/src/rs/cyclotomic_coset/test_cc_select_cosets.c:107-187
    assert _select(16, 3) == ([(257, 8), (4369, 4), (13107, 4)], [(21845, 2), (0, 1)])
    assert _select(22, 17) == ([(771, 8), (1285, 8), (30583, 4), (21845, 2)],
                               [(257, 8), (4369, 4), (13107, 4), (0, 1)])


@pytest.mark.parametrize("name,k,r", [("gmat_4_2", 4, 2), ("gmat_10_4", 10, 4), ("gmat_128_32", 128, 32),
                                      ("gmat_4096_1024", 4096, 1024)])
def test_encode_matrix_matches_reference(name, k, r):
    # golden = reference encode of unit vectors: repair word i of row p is G[p][i]
    M, ins, outs = rs_amd.coding_matrix(k, r)
    assert M.shape == (r, k) and (ins == np.arange(k)).all() and (outs == np.arange(r)).all()
    check_golden(case(name), M.astype("<u2").tobytes())


@pytest.mark.parametrize("name", ["dmat_128_32_bench", "dmat_128_32_rand"])
def test_decode_matrix_matches_reference(name):
    c = case(name)
    k, r = c["k"], c["r"]
    buf, er = case_inputs(c, 0)
    M, ins, outs = rs_amd.coding_matrix(k, r, er)
    words = buf.view("<u2").copy()  # [k+r][k+r]: unit words at the survivors
    for row, slot in enumerate(outs):
        words[slot] = 0
        words[slot, ins] = M[row]
    check_golden(c, words.astype("<u2").tobytes())


def _apply_case(c):
    """Apply the engine's matrices with numpy GF arithmetic to a golden case's inputs."""
    k, r, S = c["k"], c["r"], c["S"]
    outs_all = []
    rc = 0
    Se = S & ~1  # odd sizes: the reference's Release build codes the even prefix, written symbols end in 0
    for s in range(c["n"]):
        buf, er = case_inputs(c, s)
        W = np.ascontiguousarray(buf[:, :Se]).view("<u2")
        if c["op"] in ("encode", "encode_iota", "gmatrix"):
            if r:
                M, ins, outs = rs_amd.coding_matrix(k, r)
                W[k:] = gf_apply(M, W[:k])
                buf[k:, :Se] = W[k:].view(np.uint8)
                buf[k:, Se:] = 0
            outs_all.append(buf[k:].tobytes())
            continue
        if c["op"] == "decode":
            M, ins, outs = rs_amd.coding_matrix(k, r)
            W[k:] = gf_apply(M, W[:k])
            buf[k:, :Se] = W[k:].view(np.uint8)
            buf[k:, Se:] = 0
            buf[er] = 0
            W[er] = 0
        if c["t"] > r:
            rc = 100
        elif er[:k].any():
            M, ins, outs = rs_amd.coding_matrix(k, r, er)
            W[outs] = gf_apply(M, W[ins])
            buf[outs, :Se] = W[outs].view(np.uint8)
            buf[outs, Se:] = 0
        outs_all.append(buf.tobytes())
    return rc, b"".join(outs_all)


NP_CASES = [c["name"] for c in manifest()["cases"]
            if c["k"] * max(c["r"], 1) * c["S"] * c["n"] <= 40_000_000 and not c["name"].startswith("gmat")
            and c["op"] not in EXTRA_OPS]


@pytest.mark.parametrize("name", NP_CASES)
def test_matrix_apply_equals_reference(name):
    """The engine's linear maps reproduce every golden vector (CPU emulation of what the GPU applies)."""
    c = case(name)
    rc, out = _apply_case(c)
    assert rc == c["rc"]
    check_golden(c, out)


def test_gf256_coordinate_arithmetic():
    """The m <= 8 kernels' arithmetic: L (alpha basis -> GF(256)^2 bytes), multiplication of a byte by a
    GF(256) coefficient through gamma-multiples and nibble tables, L^-1 -- equals field multiplication."""
    lbyte, ibyte, red = rs_amd.gamma_tables()
    assert red == 0x1D
    exp, log = gf_tables()
    rng = np.random.default_rng(7)
    x = rng.integers(0, 65536, 4096).astype(np.int64)
    L = lbyte[0][x & 255].astype(np.int64) ^ lbyte[1][x >> 8]

    def xt(b):
        return ((b << 1) & 0xFE) ^ np.where(b & 0x80, red, 0)

    for e in rng.integers(0, 255, 64):
        c = int(exp[257 * int(e)])  # a GF(256) element
        cb = int(lbyte[0][c & 255] ^ lbyte[1][c >> 8])
        assert cb < 256
        m = [L & 0xFF, L >> 8]
        mult = [[mm] for mm in m]
        for j in range(1, 8):
            for h in range(2):
                mult[h].append(xt(mult[h][-1]))
        prod = [np.zeros_like(x), np.zeros_like(x)]
        for h in range(2):
            for j in range(8):
                if cb >> j & 1:
                    prod[h] ^= mult[h][j]
        u = prod[0] | (prod[1] << 8)
        y = ibyte[0][u & 255].astype(np.int64) ^ ibyte[1][u >> 8]
        want = np.where(x == 0, 0, exp[(log[c] + log[x]) % 65535])
        assert (y == want).all()


def test_jit_precompile_offline(tmp_path, monkeypatch):
    """The hiprtc specialiser generates and compiles a gfx950 code object without a GPU."""
    monkeypatch.setenv("RS_AMD_JIT_CACHE", str(tmp_path))
    rs_amd.jit_precompile(10, 4)
    er = rs_amd.bench_pattern(10, 4)
    rs_amd.jit_precompile(10, 4, er)
    files = list(tmp_path.glob("*.co"))
    assert len(files) == 2 and all(f.stat().st_size > 1000 for f in files)


def test_invalid_arguments():
    with pytest.raises(rs_amd.RSError) as e:
        rs_amd.coding_matrix(65000, 1000)
    assert e.value.rc == rs_amd.RS_ERR_INVALID
    er = np.zeros(6, bool)
    er[:3] = True
    with pytest.raises(rs_amd.RSError) as e:
        rs_amd.coding_matrix(4, 2, er)
    assert e.value.rc == rs_amd.RS_ERR_CANNOT_RESTORE


def test_release_build_has_no_ablation_kernels():
    """Timing ablations (wrong results by construction) live only in the diagnostic build
    (make diag -> librs_amd_diag.so); the product library must not contain them."""
    import subprocess
    out = subprocess.run(["nm", "-C", rs_amd.LIB_PATH], capture_output=True, text=True, check=True).stdout
    for bad in ("k_apply_m8_lds<1", "k_apply_m8_lds<2", "k_apply_m8_lds<3", "k_apply_m8_lds<4", "k_apply_m8_lds<6",
                "k_apply_m8_lds<0, true>", "k_apply_m8_v1<1>", "k_apply_m16_v1<1>", "k_apply_m8_idx<4, 4>"):
        assert bad not in out, bad
    assert "DIAGNOSTIC" not in rs_amd.version()


REF_INC = "/root/reference/include"
LAYOUT_C = r"""
#include <stddef.h>
#include <stdio.h>
#include <memory/seq.h>
#include <memory/symbol.h>
#include <rs/cyclotomic_coset.h>
#include <rs/fft.h>
#include <rs/gf65536.h>
#include <rs/reed_solomon.h>
int main(void) {
    printf("%zu %zu %zu %zu %zu\n", sizeof(GF_t), offsetof(GF_t, log_table), offsetof(GF_t, normal_bases),
           offsetof(GF_t, normal_repr_by_subfield), offsetof(GF_t, _normal_repr_by_subfield_memory));
    printf("%zu %zu %zu %zu\n", sizeof(CC_t), sizeof(coset_t), sizeof(symbol_t), sizeof(symbol_seq_t));
    printf("%zu %zu %zu\n", offsetof(RS_t, gf), offsetof(RS_t, cc), offsetof(symbol_seq_t, symbols));
    printf("%d %d %d %d %d\n", N, GF_FIELD_SIZE, GF_PRIMITIVE_POLY, RS_ERR_CANNOT_RESTORE, RS_COSET_LOCATOR_MAX_LEN);
    return 0;
}
"""


def test_header_layouts_match_reference(tmp_path):
    """The public structs and constants have the reference's layout and values (compiled once against
    the reference's headers, once against this repo's); needs /root/reference (this container)."""
    import subprocess
    if not os.path.isdir(REF_INC):
        pytest.skip("reference headers absent")
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    outs = []
    for inc in (REF_INC, os.path.join(REPO, "include")):
        exe = tmp_path / ("ref" if inc == REF_INC else "ours")
        subprocess.check_call(["gcc", "-std=c11", "-w", f"-I{inc}", "-o", str(exe), str(src)])
        outs.append(subprocess.check_output([str(exe)], text=True))
    assert outs[0] == outs[1], outs


def test_seq_create_without_gpu_falls_back_to_heap():
    """seq_create of a large sequence tries a page-locked arena; with no GPU (this container) it falls
    back to zeroed heap symbols, and seq_destroy / symbol_destroy free either kind."""
    q = rs_amd.Seq(160, 65536 + 2)
    assert all(s.size == 65538 and not s.any() for s in q.symbols)
    q.symbols[3][:] = 7
    v = q.view(128, 32)
    assert v.length == 32 and v.symbol_size == 65538
    q.close()
    small = rs_amd.Seq(4, 16)  # below the arena threshold: always heap
    assert len(small.symbols) == 4
    small.close()


def test_symbol_create_pages_and_pool():
    """symbol_create from 16 KiB (seq_create with RS_AMD_PINNED_SEQ=0): whole zeroed pages of their own at
    increasing addresses (consecutive symbols of one size at one stride, the zero-copy condition), and no
    HIP call (registration waits for the first rs_* call that moves the symbol: 0, never -1);
    symbol_destroy parks them in the idle pool and the next symbols of that size take the same addresses
    back, zeroed, so a once-registered address never returns to other allocators."""
    S = 3 * 4096 + 4096 + 100
    st0 = rs_amd.symbol_stats()
    os.environ["RS_AMD_PINNED_SEQ"] = "0"
    try:
        q = rs_amd.Seq(6, S)
        addrs = [x.ctypes.data for x in q.symbols]
        page = (S + 4095) // 4096 * 4096
        assert all(a % 4096 == 0 for a in addrs)
        assert [b - a for a, b in zip(addrs, addrs[1:])] == [page] * 5
        assert all(rs_amd.symbol_registered(x) == 0 for x in q.symbols)
        for x in q.symbols:
            x[:] = 0xA5
        q.close()
        q2 = rs_amd.Seq(6, S)
        assert sorted(x.ctypes.data for x in q2.symbols) == sorted(addrs)
        assert all(not x.any() for x in q2.symbols)
        q2.close()
    finally:
        os.environ.pop("RS_AMD_PINNED_SEQ")
    st1 = rs_amd.symbol_stats()
    assert st1["registrations"] == st0["registrations"] and st1["register_failures"] == st0["register_failures"]
    assert st1["idle_reuses"] - st0["idle_reuses"] == 6
    small = rs_amd.Seq(3, 4096)  # below 16 KiB: calloc, not tracked
    assert all(rs_amd.symbol_registered(x) == -1 for x in small.symbols)
    small.close()


def _maps_perms(addr):
    """Permissions of the /proc/self/maps mapping holding addr (None when unmapped)."""
    with open("/proc/self/maps") as f:
        for line in f:
            lo, hi = (int(v, 16) for v in line.split()[0].split("-"))
            if lo <= addr < hi:
                return line.split()[1]
    return None


def test_symbol_churn_pool_cap_and_reservations():
    """Allocator churn of library-allocated symbol pages (rs_hostmem.cpp), the code of the round-3 fault:
    random sizes 16 KiB .. 200 KiB, random destroy order, a small idle-pool cap. Live counts return to the
    baseline, the pool never exceeds its cap, blocks destroyed past it are retired (memory returned:
    PROT_NONE, address kept reserved) and no retired address is handed out again; a parked address comes
    back only through the pool. Under tests/test_sanitizers.py (RS_AMD_SYM_VA_MB=1) the churn also
    crosses many address reservations (sym_va_take)."""
    rng = np.random.default_rng(11)
    old_cap = rs_amd.symbol_pool_cap(3 << 20)
    st0 = rs_amd.symbol_stats()
    retired, seen = set(), set()
    live = []
    os.environ["RS_AMD_PINNED_SEQ"] = "0"
    try:
        for it in range(60):
            n = int(rng.integers(1, 9))
            S = int(rng.integers(16 << 10, 200 << 10))
            q = rs_amd.Seq(n, S)
            for x in q.symbols:
                a = x.ctypes.data
                assert a % 4096 == 0 and not x.any()
                assert a not in retired, "a retired address was handed out again"
                assert rs_amd.symbol_registered(x) == 0
                x[:] = it & 0xFF
                seen.add(a)
            live.append(q)
            if len(live) > 4 or rng.integers(0, 2):
                victim = live.pop(int(rng.integers(0, len(live))))
                before = rs_amd.symbol_stats()
                addrs = [x.ctypes.data for x in victim.symbols]
                victim.close()
                after = rs_amd.symbol_stats()
                assert after["idle_bytes"] <= (3 << 20)
                if after["retired_blocks"] > before["retired_blocks"]:
                    # every block of the victim not parked was retired: its pages are PROT_NONE now
                    gone = [a for a in addrs if _maps_perms(a) == "---p"]
                    assert len(gone) == after["retired_blocks"] - before["retired_blocks"]
                    retired.update(gone)
        for q in live:
            q.close()
    finally:
        os.environ.pop("RS_AMD_PINNED_SEQ")
        rs_amd.symbol_pool_cap(old_cap)
    st1 = rs_amd.symbol_stats()
    assert st1["live"] == st0["live"]
    assert st1["retired_blocks"] > st0["retired_blocks"] and st1["idle_reuses"] > st0["idle_reuses"]
    assert st1["unregister_failures"] == st0["unregister_failures"] and st1["stuck_blocks"] == st0["stuck_blocks"]
    assert len(retired) > 0


def test_bench_traffic_lookup_is_per_leg(tmp_path, monkeypatch):
    """bench.py's PMC traffic lookup (profiles/traffic.json) keys records by leg: the GF(2^16) route runs
    kernels of one name on both legs ("cs16t+bs16"), whose HBM bytes differ; the newest record wins."""
    import json
    import sys
    sys.path.insert(0, REPO)
    import bench
    cfg = "k4096_r1024_S1024_n1024_t1024"
    name = "kern[route]"  # a bracketed (content-addressed) name: no source-hash check
    recs = [dict(leg="decode", bench_kernel=name, config=cfg, traffic_bytes=3.0),
            dict(leg="encode", bench_kernel=name, config=cfg, traffic_bytes=1.0),
            dict(leg="encode", bench_kernel=name, config=cfg, traffic_bytes=2.0)]
    path = tmp_path / "traffic.json"
    path.write_text(json.dumps({"records": recs}))
    monkeypatch.setattr(bench, "TRAFFIC_JSON", str(path))
    assert bench.measured_traffic(name, cfg, leg="encode") == 2
    assert bench.measured_traffic(name, cfg, leg="decode") == 3
    assert bench.measured_traffic("other[k]", cfg, leg="encode") is None


def _regs(tok):
    """Register numbers named by an operand: ('s', {..}) / ('v', {..}) or None."""
    m = re.fullmatch(r"([sv])(\d+)", tok)
    if m:
        return m.group(1), {int(m.group(2))}
    m = re.fullmatch(r"([sv])\[(\d+):(\d+)\]", tok)
    if m:
        return m.group(1), set(range(int(m.group(2)), int(m.group(3)) + 1))
    return None


def test_no_compiler_code_touches_in_flight_load_registers(tmp_path):
    """k_cs16 / k_bs16 issue scalar and vector loads inside one step's asm statement that land in
    registers the NEXT step reads (records, slot offsets, inputs); k_cs16t keeps its whole loop in one
    statement. Compiler-generated code between the asm statements must never read or write a register a
    load issued by an earlier statement may still be filling (the round-3 k_cs16t bug: slot offsets copied
    before their s_load landed). Loads and waits are tracked through the asm text of the gfx950 assembly
    of rs_kernels.hip (s_waitcnt lgkmcnt(0) / vmcnt(0) retire the scalar / vector loads)."""
    import subprocess
    pkg = os.path.join(REPO, "reed-solomon_amd")
    out = tmp_path / "k.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                           "-I../include", "-Icsrc", "--cuda-device-only", "-S", "csrc/rs_kernels.hip", "-o", str(out)],
                          cwd=pkg, stderr=subprocess.DEVNULL)
    text = out.read_text().splitlines()
    for sym in ("_ZN5rsamd6k_cs16ENS_8Cs16ArgsE", "_ZN5rsamd6k_bs16ENS_8Cs16ArgsE", "_ZN5rsamd7k_cs16tENS_8Cs16ArgsE"):
        start = next(i for i, ln in enumerate(text) if ln.startswith(sym + ":"))
        end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
        pend = {"s": set(), "v": set()}
        inside, checked = False, 0
        for raw in text[start:end]:
            if ";;#ASMSTART" in raw or ";;#ASMEND" in raw:
                inside = ";;#ASMSTART" in raw
                continue
            ln = raw.split(";")[0].strip()
            if not ln or ln.endswith(":") or ln.startswith("."):
                continue
            op, _, rest = ln.partition(" ")
            ops = [x.strip().split()[0] for x in re.split(r",\s*(?![^\[]*\])", rest) if x.strip()] if rest else []
            if inside:  # the asm's own loads and waits
                if op == "s_waitcnt":
                    if "lgkmcnt(0)" in rest:
                        pend["s"].clear()
                    if "vmcnt(0)" in rest:
                        pend["v"].clear()
                elif op.startswith(("s_load_dword", "buffer_load_dword", "global_load_dword")) and ops:
                    r = _regs(ops[0])
                    if r:
                        pend[r[0]] |= r[1]
                continue
            checked += 1
            for tok in ops:
                r = _regs(tok)
                assert not (r and r[1] & pend[r[0]]), (sym, raw)
        assert checked > 0


@pytest.mark.parametrize("k,r,t_info,t_rep", [(10, 4, 3, 1), (120, 32, 32, 0), (300, 64, 40, 24), (40, 20, 7, 13)])
def test_reencode_solve_is_the_inverse_cauchy(k, r, t_info, t_rep):
    """The closed form behind both per-stripe re-encode plans (k_plan_reenc_m8, k_plan16_reenc_rec):
    with E the erased information slots, R' the first |E| surviving repair slots and T = E + (repair slots
    not in R'), W'[p][q] = L_T(X_q) / ((X_q + X_p) L_T'(X_p)) inverts G[R', E] (G = the encode matrix from
    the oracle, reed_solomon.c:338-441), so W' S'_R' recovers the erased information from the re-encode
    differences. Checked over GF(2^16) on CPU; GF(256) codes (k + r <= 255) included."""
    from _util import oracle_encode, oracle_positions
    exp, log = gf_tables()
    N = 65535
    X = exp[oracle_positions(k, r).astype(np.int64)]
    # G[:, Q] = the repair words of the unit information vector e_Q (one 2-byte word per symbol)
    G = np.zeros((r, k), np.uint16)
    for q in range(k):
        buf = np.zeros((k + r, 2), np.uint8)
        buf[q, 0] = 1
        assert oracle_encode(k, r, buf) == 0
        G[:, q] = buf[k:, 0].astype(np.uint16) | (buf[k:, 1].astype(np.uint16) << 8)
    rng = np.random.default_rng(k * 7 + t_info)
    E = np.sort(rng.choice(k, t_info, replace=False))
    rep_er = np.sort(rng.choice(r, t_rep, replace=False)) + k
    surv = [s for s in range(k, k + r) if s not in set(rep_er)]
    Rp = np.array(surv[:t_info])
    T = np.array(list(E) + [s for s in range(k, k + r) if s not in set(Rp)], dtype=np.int64)
    assert len(T) == r

    def logsum(x, excl=None):
        return sum(int(log[int(x ^ X[e])]) for e in T if e != excl) % N

    W = np.zeros((t_info, t_info), np.uint16)
    for i, p in enumerate(E):
        lr = logsum(X[p], excl=p)
        for j, q in enumerate(Rp):
            W[i, j] = exp[(logsum(X[q]) + 2 * N - lr - int(log[int(X[p] ^ X[q])])) % N]
    prod = gf_apply(W, G[Rp - k][:, E])
    assert np.array_equal(prod, np.eye(t_info, dtype=np.uint16))


@pytest.mark.parametrize("value,want", [(None, 0), ("0", 0), ("1", 1)])
def test_checked_launch_mode_switch(value, want):
    """RS_AMD_CHECK (rsg_check_enabled): read once per process, so each setting runs in a fresh one."""
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("RS_AMD_CHECK", None)
    if value is not None:
        env["RS_AMD_CHECK"] = value
    code = ("import sys; sys.path.insert(0, %r); import rs_amd; print(rs_amd._lib.rsg_check_enabled())"
            % os.path.join(REPO, "reed-solomon_amd"))
    out = subprocess.check_output([sys.executable, "-c", code], env=env, text=True)
    assert out.strip().splitlines()[-1] == str(want)


def test_symbol_ops_validation_without_gpu():
    """rsg_symbol_ops rejects a batch before anything is queued (RS_ERR_INVALID, no device touched): an
    unknown op, a null or misaligned pointer, overlapping targets, a source that is another op's target
    (chains run side by side). An empty batch, or one of zero-word symbols, is a no-op (rc 0)."""
    A, B, C = 0x10000, 0x20000, 0x30000  # fake 4-byte aligned addresses: never dereferenced here
    S = 4096
    inval = [
        [(3, A, B, 1)],                                    # unknown op
        [(rs_amd.OP_ADD, 0, B, 0)],                        # null target
        [(rs_amd.OP_MADD, A, 0, 5)],                       # null source
        [(rs_amd.OP_ADD, A + 2, B, 0)],                    # misaligned target
        [(rs_amd.OP_MADD, A, B + 1, 7)],                   # misaligned source
        [(rs_amd.OP_ADD, A, B, 0), (rs_amd.OP_ADD, A + S - 4, C, 0)],  # overlapping targets
        [(rs_amd.OP_ADD, A, B, 0), (rs_amd.OP_MADD, C, A, 9)],        # reads another chain's target
        [(rs_amd.OP_ADD, A, B, 0), (rs_amd.OP_MADD, C, A + 100, 9)],  # reads inside another chain's target
        [(rs_amd.OP_MUL, B, 0, 3), (rs_amd.OP_ADD, A, B - S + 2, 0)],  # source overlaps a target's start
    ]
    for ops in inval:
        assert rs_amd.symbol_ops(ops, S, stream=0, check=False) == rs_amd.RS_ERR_INVALID, ops
    assert rs_amd.symbol_ops([], S, stream=0) == 0
    assert rs_amd.symbol_ops([(rs_amd.OP_ADD, A, B, 0)], 1, stream=0) == 0  # no whole word: nothing to do


def test_traffic_composite_legs_and_component_split(tmp_path):
    """scripts/traffic.py on synthetic rocprofv3 counter CSVs: composite legs (the GF(2^16) route's
    cs16t + bs16) are cut out of the dispatch order encode / decode alternately, summed per launch, and split
    per component kernel; a stray dispatch at a leg boundary (a dense first launch) is skipped."""
    import csv
    import sys as _sys
    _sys.path.insert(0, os.path.join(REPO, "scripts"))
    import traffic
    d = tmp_path / "f"
    d.mkdir()
    rows = [(1, "rsamd::k_bs16(x)", 5.0),  # boundary stray: skipped
            (2, "rsamd::k_cs16t(x)", 100.0), (3, "rsamd::k_bs16(x)", 10.0),   # encode 1
            (4, "rsamd::k_cs16t(x)", 300.0), (5, "rsamd::k_bs16(x)", 30.0),   # decode 1
            (6, "rsamd::k_cs16t(x)", 110.0), (7, "rsamd::k_bs16(x)", 12.0),   # encode 2
            (8, "rsamd::k_cs16t(x)", 290.0), (9, "rsamd::k_bs16(x)", 31.0)]   # decode 2
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for did, name, v in rows:
            for half in (0.5, 0.5):  # counters come per XCD / SE: summed per dispatch
                w.writerow({"Dispatch_Id": did, "Kernel_Name": name, "Counter_Name": "FETCH_SIZE", "Counter_Value": v * half})
    out = traffic.per_leg_composite(str(d), "FETCH_SIZE", {"encode": ["cs16t", "bs16"], "decode": ["cs16t", "bs16"]})
    assert [t for t, _ in out["encode"]] == [110.0, 122.0]
    assert [t for t, _ in out["decode"]] == [321.0, 330.0]
    assert out["decode"][0][1] == {"cs16t": 290.0, "bs16": 31.0}


def test_traffic_merge_replaces_by_key_and_bench_finds_the_record(tmp_path):
    """scripts/traffic_merge.py folds a traffic.py run into the PMC table: a record with the same (leg, kernel,
    config, source hash) replaces the old one, others are kept; bench.measured_traffic then reads it for a
    JIT kernel name (content-addressed, no source-hash check)."""
    import importlib.util
    import json

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod
    tm = load("traffic_merge", os.path.join(REPO, "scripts", "traffic_merge.py"))
    rec = lambda leg, b, h="h0": {"leg": leg, "bench_kernel": "rs_xj[4x10:abc]", "config": "k10_r4_S4096_n1024_t4",
                                   "src_hash": h, "traffic_bytes": b}
    table = tmp_path / "traffic.json"
    table.write_text(json.dumps({"records": [rec("encode", 1), rec("decode", 2)]}))
    run = tmp_path / "run.json"
    run.write_text(json.dumps({"records": [rec("encode", 10), rec("encode", 30, "h1")]}))
    tm.main([str(run)], table=str(table))
    recs = json.loads(table.read_text())["records"]
    assert sorted((r["leg"], r["src_hash"], r["traffic_bytes"]) for r in recs) == \
        [("decode", "h0", 2), ("encode", "h0", 10), ("encode", "h1", 30)]
    bench = load("bench_for_traffic", os.path.join(REPO, "bench.py"))
    bench.TRAFFIC_JSON = str(table)
    assert bench.measured_traffic("rs_xj[4x10:abc]", "k10_r4_S4096_n1024_t4", leg="encode") == 30  # newest wins
    assert bench.measured_traffic("rs_xj[4x10:abc]", "k10_r4_S4096_n1024_t4", leg="decode") == 2
    assert bench.measured_traffic("rs_xj[4x10:abc]", "k10_r4_S4096_n1024_t1", leg="decode") is None
