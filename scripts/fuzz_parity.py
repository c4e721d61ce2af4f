"""Randomised parity fuzz on the GPU against the CPU oracle (TEST INFRASTRUCTURE): random (k, r),
symbol sizes with and without tail columns, stripe counts and erasure patterns, through every kernel
path: matrix-specialised XOR kernels (jit=1), generic GF(256) kernels (jit=0), GF(2^16) codes
(hand-scheduled kernel, split-K on small grids, device-built plans), and rsg_decode_batch with a
pattern per stripe (device-built plans; for GF(2^16) codes, "batch16", one plan rebuilt on the stream
per pattern), the GF(2^16) syndrome route ("route": k_cs16 + k_bs16 / second stage) and the per-call
drop-in API on seq_create arenas ("dropin"). Prints one JSON line per case and a summary.
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

rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 2024)
budget = float(sys.argv[2]) if len(sys.argv) > 2 else 240.0
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


def one(family):
    if family == "dropin":
        return one_dropin()
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
    codec = rs_amd.Codec(k, r, **kw)
    if family in ("route", "reenc"):
        codec.set_option("m16_route_min_bytes", 0)  # decode patterns on the route at once
        codec.set_option("m16_cs_col", int(rng.choice([256, 1024])))  # route kernels' block layout
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


families = sys.argv[3].split(",") if len(sys.argv) > 3 else ["xj", "generic", "m16", "route", "reenc", "batch",
                                                             "batch16", "dropin"]
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
