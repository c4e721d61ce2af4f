"""Randomised parity fuzz on the GPU against the CPU oracle (TEST INFRASTRUCTURE): random (k, r),
symbol sizes with and without tail columns, stripe counts and erasure patterns, through every kernel
path: matrix-specialised XOR kernels (jit=1), generic GF(256) kernels (jit=0), GF(2^16) codes
(hand-scheduled kernel, split-K on small grids, device-built plans), and rsg_decode_batch with a
pattern per stripe (device-built plans; for GF(2^16) codes, "batch16", one plan rebuilt on the stream
per pattern), the GF(2^16) syndrome route ("route": k_cs16 + k_bs16 / second stage), the per-call
drop-in API on seq_create arenas ("dropin"); round 3: the per-stripe GF(2^16) route ("ps16"), decode
patterns closed under a Frobenius power ("orbit": the k_bs16 stage over row orbits) and the per-call API
on registered symbol_create buffers ("dropin_reg"); round 6: batched symbol ops (rsg_symbol_ops, "symops"). Prints one JSON line per case and a summary.
usage: fuzz_parity.py [seed] [seconds] [family,family,...]"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "reed-solomon_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import rs_amd  # noqa: E402
from _util import oracle_decode, oracle_encode  # noqa: E402

rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 and __name__ == "__main__" else 2024)
budget = float(sys.argv[2]) if len(sys.argv) > 2 and __name__ == "__main__" else 240.0
t_end = time.time() + budget
counts = {}
fails = 0


def one_dropin():
    """Reference per-call API on library-allocated (seq_create) stripes: page-locked arenas, DMA in
    place, zero-copy XOR-kernel launches once a plan is specialised; 4 restores of one pattern."""
    if rng.integers(0, 2):
        k = int(rng.integers(20, 200))
        r = int(rng.integers(1, min(255 - k, 64) + 1))
    else:
        k = int(rng.integers(200, 700))
        r = int(rng.integers(max(1, 256 - k), 200))
    if rng.integers(0, 2):  # slab-allocated small stripe: zero-copy launches of any kernel
        S = 2 * int(rng.integers(1, max(2, (1 << 19) // (k + r))))
    else:
        lo = max(1024, (1 << 20) // (2 * (k + r)))
        S = 2 * int(rng.integers(lo, max(16384, lo + 1024)))
    q = rs_amd.Seq(k + r, S)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    for i in range(k):
        q.symbols[i][:] = data[i]
    rs = rs_amd.RS()
    want = np.zeros((k + r, S), np.uint8)
    want[:k] = data
    assert oracle_encode(k, r, want) == 0
    ok = True
    er = np.zeros(k + r, bool)
    er[rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    for call in range(4):
        assert rs.generate_repair_symbols(q, r) == 0
        ok = ok and bool(np.array_equal(np.stack(q.symbols), want))
        for i in np.nonzero(er)[0]:
            q.symbols[i][:] = 0
        assert rs.restore_symbols(k, r, q, er, int(er.sum())) == 0
        got = np.stack(q.symbols)
        ok = ok and bool(np.array_equal(got[:k], data)) and not got[k:][er[k:]].any()
    pitch = q.symbols[1].ctypes.data - q.symbols[0].ctypes.data if k + r > 1 else 0
    q.close()
    rs.close()
    return dict(family="dropin", k=k, r=r, S=S, stripes=1, t=int(er.sum()), arena=pitch == (S + 15) // 16 * 16, ok=ok)


def one_dropin_reg():
    """Per-call API on separately allocated symbols (RS_AMD_PINNED_SEQ=0: symbol_create per symbol, from
    16 KiB page-aligned, page-locked on first use): zero-copy kernels when the symbols sit at one stride,
    else gather / scatter kernels over the symbol pointers; GF(256) and GF(2^16) codes."""
    if rng.integers(0, 2):
        k = int(rng.integers(20, 200))
        r = int(rng.integers(1, min(255 - k, 64) + 1))
    else:
        k = int(rng.integers(200, 600))
        r = int(rng.integers(max(1, 256 - k), 150))
    S = 16 * int(rng.integers(1024, 4096 + 1))  # 16 .. 64 KiB, multiples of 16
    os.environ["RS_AMD_PINNED_SEQ"] = "0"
    try:
        q = rs_amd.Seq(k + r, S)
    finally:
        os.environ.pop("RS_AMD_PINNED_SEQ")
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    for i in range(k):
        q.symbols[i][:] = data[i]
    rs = rs_amd.RS()
    want = np.zeros((k + r, S), np.uint8)
    want[:k] = data
    assert oracle_encode(k, r, want) == 0
    ok = True
    registered = None
    er = np.zeros(k + r, bool)
    er[rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    for call in range(4):
        assert rs.generate_repair_symbols(q, r) == 0
        if registered is None:  # registration happens on first use (round 4: symbol_create makes no HIP call)
            registered = all(rs_amd.symbol_registered(x) == 1 for x in q.symbols)
            ok = registered
        ok = ok and bool(np.array_equal(np.stack(q.symbols), want))
        for i in np.nonzero(er)[0]:
            q.symbols[i][:] = 0
        assert rs.restore_symbols(k, r, q, er, int(er.sum())) == 0
        got = np.stack(q.symbols)
        ok = ok and bool(np.array_equal(got[:k], data)) and not got[k:][er[k:]].any()
    q.close()
    rs.close()
    return dict(family="dropin_reg", k=k, r=r, S=S, stripes=1, t=int(er.sum()), registered=registered, ok=ok)


def one_ps16():
    """rsg_decode_batch of a GF(2^16) code with a different pattern on every stripe: the per-stripe route
    (syndromes of all slots + a device-built solve per stripe); garbage in erased slots."""
    k = int(rng.integers(150, 700))
    r = int(rng.integers(max(1, 256 - k), 300))
    S = 1024 * int(rng.integers(1, 5))
    n = int(rng.integers(3, 40))
    dev = torch.zeros((n, k + r, S), dtype=torch.uint8, device="cuda")
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev.copy_(torch.from_numpy(host))
    codec = rs_amd.Codec(k, r)
    codec.encode(dev)
    torch.cuda.synchronize()
    full = dev.cpu().numpy()
    pats = np.zeros((n, k + r), bool)
    for s in range(n):
        pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
    rcv = full.copy()
    rcv[pats] = rng.integers(0, 256, (int(pats.sum()), S), dtype=np.uint8)
    dev.copy_(torch.from_numpy(rcv))
    assert codec.decode_batch(dev, pats) == 0
    torch.cuda.synchronize()
    out = dev.cpu().numpy()
    ok = bool(np.array_equal(out[:, :k], full[:, :k]))
    rep = pats.copy()
    rep[:, :k] = False
    ok = ok and bool(np.array_equal(out[rep], rcv[rep]))
    for s in rng.choice(n, min(n, 3), replace=False):
        ref = rcv[s].copy()
        ref[pats[s]] = 0
        assert oracle_decode(k, r, ref, pats[s], int(pats[s].sum())) == 0
        ok = ok and bool(np.array_equal(out[s, :k], ref[:k]))
    kern = codec.last_kernel
    codec.close()
    return dict(family="ps16", k=k, r=r, S=S, stripes=n, decode=kern, ok=ok)


def one_orbit():
    """GF(2^16) decode patterns closed under a Frobenius power (runs of slots spaced 16 / 2^j apart inside
    the 16-slot cosets, whole cosets, like the C5 bench pattern): the plain route with the k_bs16 stage
    over row orbits; repair cosets or parts of them may be erased too."""
    k = 16 * int(rng.integers(20, 90))
    r = 16 * int(rng.integers(4, 18))
    S = 1024 * int(rng.integers(1, 3))
    n = int(rng.integers(1, 3))
    from _util import oracle_positions
    pos = oracle_positions(k, r).astype(np.int64)
    runs, i = [], 0
    while i < k + r:  # cosets: runs of slots whose positions double
        j = i + 1
        while j < k + r and j - i < 16 and pos[j] == (2 * pos[j - 1]) % 65535:
            j += 1
        runs.append((i, j - i))
        i = j
    step = int(rng.choice([1, 2, 4, 8]))  # slot spacing inside a coset: orbit under x -> x^(2^step)
    er = np.zeros(k + r, bool)
    for a, m in [runs[x] for x in rng.permutation(len(runs))]:
        if m != 16:
            continue
        c = int(rng.integers(0, step))
        sl = [a + c + step * b for b in range(16 // step)]
        if er.sum() + len(sl) > r:
            break
        er[sl] = True
    if not er[:k].any():
        return dict(family="orbit", k=k, r=r, S=S, stripes=n, skipped=True, ok=True)
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
    dev.copy_(torch.from_numpy(poisoned))
    codec.decode(dev, er)
    torch.cuda.synchronize()
    out = dev.cpu().numpy()
    ok = True
    for s in range(n):
        ref = poisoned[s].copy()
        assert oracle_decode(k, r, ref, er, int(er.sum())) == 0
        ok = ok and bool(np.array_equal(out[s], ref))
    kern = codec.last_kernel
    codec.close()
    return dict(family="orbit", k=k, r=r, S=S, stripes=n, t=int(er.sum()), step=step, decode=kern, ok=ok)


def one_symops():
    """rsg_symbol_ops: random chains of gf_add / gf_mul / gf_madd (coefficients 0, 1 and general, sources equal
    to their own target) over random symbol sizes (odd word counts, odd byte counts), against the ops applied
    one after another with numpy (GF(2^16) exp / log tables)."""
    from _util import gf_tables
    exp, log = gf_tables()
    S = int(rng.choice([2, 6, 9, 1024, 1030, 4096, 65536])) + 2 * int(rng.integers(0, 8)) * int(rng.integers(0, 2))
    n_t, n_s = int(rng.integers(1, 40)), int(rng.integers(1, 40))
    P = (S + 15) // 16 * 16
    host = rng.integers(0, 256, (n_t + n_s, P), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    addr = [dev[i].data_ptr() for i in range(n_t + n_s)]
    ops = []
    for _ in range(int(rng.integers(1, 400))):
        t = int(rng.integers(n_t))
        kind = int(rng.choice([0, 1, 2], p=[0.2, 0.1, 0.7]))
        src = t if rng.random() < 0.05 else n_t + int(rng.integers(n_s))
        coef = int(rng.choice([0, 1, int(rng.integers(2, 65536))], p=[0.05, 0.05, 0.9]))
        ops.append((kind, addr[t], addr[src], coef))
    rs_amd.symbol_ops(ops, S)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    nw = S // 2
    want = host.copy()
    idx = {a: i for i, a in enumerate(addr)}
    for kind, a, b, c in ops:
        wa = want[idx[a], :2 * nw].view("<u2").astype(np.int64)
        x = wa if kind == 1 else want[idx[b], :2 * nw].view("<u2").astype(np.int64)
        y = x if (kind == 0 or (kind == 2 and c == 1)) else (
            np.where(x != 0, exp[(log[x] + log[c]) % 65535], 0) if c else np.zeros_like(x))
        if kind == 1 and c == 1:
            y = x
        wa = y if kind == 1 else wa ^ y
        want[idx[a], :2 * nw] = wa.astype("<u2").view(np.uint8)
    return dict(family="symops", S=S, targets=n_t, sources=n_s, ops=len(ops), ok=bool(np.array_equal(got, want)))


def one(family):
    if family == "symops":
        return one_symops()
    if family == "dropin":
        return one_dropin()
    if family == "dropin_reg":
        return one_dropin_reg()
    if family == "ps16":
        return one_ps16()
    if family == "orbit":
        return one_orbit()
    if family in ("xj", "generic", "batch"):
        k = int(rng.integers(1, 200))
        r = int(rng.integers(1, min(255 - k, 80) + 1))
    elif family == "m16":
        k = int(rng.integers(200, 1500))
        r = int(rng.integers(max(1, 256 - k), 300))
    elif family == "route":  # GF(2^16) syndrome route: K, R >= 64, whole 1 KiB column chunks
        k = int(rng.integers(200, 1200))
        r = int(rng.integers(max(64, 256 - k), 300))
    elif family == "reenc":  # re-encode decode: information erasures only, t >= 0.9 r
        k = int(rng.integers(300, 1500))
        r = int(rng.integers(max(64, 256 - k), 300))
    else:  # batch16: GF(2^16) codes, small enough for the oracle to check every stripe quickly
        k = int(rng.integers(150, 500))
        r = int(rng.integers(max(1, 256 - k), 160))
    S = int(rng.choice([2048, 4096, 8192, 1024])) + 8 * int(rng.integers(0, 64)) * int(rng.integers(0, 2))
    if family in ("m16", "batch16"):
        S = min(S, 4096 if family == "m16" else 2048)
    if family in ("route", "reenc"):
        S = 1024 * int(rng.integers(1, 4))
    n = int(rng.integers(1, 5)) if family not in ("batch", "batch16") else int(rng.integers(20, 60))
    if family in ("route", "reenc"):
        n = int(rng.integers(1, 3))
    host = np.zeros((n, k + r, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    kw = {"xj": dict(jit=1), "generic": dict(jit=0), "m16": {}, "route": {}, "reenc": {}, "batch": dict(batch_plans=1),
          "batch16": dict(batch_plans=1)}[family]
    col = int(rng.choice([256, 1024])) if family in ("route", "reenc") else 256
    # the 1 KiB route block layout is a diagnostic-build option (rs_amd.diag_module())
    codec = (rs_amd.diag_module() if col == 1024 else rs_amd).Codec(k, r, **kw)
    if family in ("route", "reenc"):
        codec.set_option("m16_route_min_bytes", 0)  # decode patterns on the route at once
        codec.set_option("m16_cs_col", col)  # route kernels' block layout
    codec.encode(dev)
    torch.cuda.synchronize()
    enc_kernel = codec.last_kernel
    got = dev.cpu().numpy()
    want = host.copy()
    for s in range(n):
        assert oracle_encode(k, r, want[s]) == 0
    ok = bool(np.array_equal(got, want))
    if family in ("batch", "batch16"):
        pats = np.zeros((n, k + r), bool)
        for s in range(n):
            pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
        poisoned = got.copy()
        poisoned[pats] = 0
        dev.copy_(torch.from_numpy(poisoned))
        assert codec.decode_batch(dev, pats) == 0
    else:
        er = np.zeros(k + r, bool)
        if family == "reenc":
            er[rng.choice(k, int(rng.integers((9 * r + 9) // 10, r + 1)), replace=False)] = True
        else:
            lo = 64 if family == "route" and rng.integers(0, 2) else 1  # t >= 64: the decode route too
            er[rng.choice(k + r, int(rng.integers(min(lo, r), r + 1)), replace=False)] = True
        pats = np.broadcast_to(er, (n, k + r))
        poisoned = got.copy()
        poisoned[:, er] = 0
        dev.copy_(torch.from_numpy(poisoned))
        codec.decode(dev, er)
    torch.cuda.synchronize()
    dec_kernel = codec.last_kernel
    out = dev.cpu().numpy()
    for s in range(n):
        ref = poisoned[s].copy()
        assert oracle_decode(k, r, ref, pats[s], int(pats[s].sum())) == 0
        ok = ok and bool(np.array_equal(out[s], ref))
    codec.close()
    return dict(family=family, k=k, r=r, S=S, stripes=n, encode=enc_kernel, decode=dec_kernel, ok=ok)


if __name__ == "__main__":
    families = sys.argv[3].split(",") if len(sys.argv) > 3 else ["xj", "generic", "m16", "route", "reenc", "batch",
                                                                 "batch16", "dropin", "ps16", "orbit", "dropin_reg", "symops"]
    i = 0
    while time.time() < t_end:
        fam = families[i % len(families)]
        i += 1
        res = one(fam)
        counts[fam] = counts.get(fam, 0) + 1
        fails += 0 if res["ok"] else 1
        print(json.dumps(res), flush=True)
    print(json.dumps({"summary": True, "cases": counts, "failures": fails}), flush=True)
    sys.exit(1 if fails else 0)
