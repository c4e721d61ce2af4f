"""Per-call latency of the reference API at C5 (k=4096, r=1024, 1 KiB symbols, one stripe per call):
encode, decode with the same erasure pattern every call (plan cached) and with a new pattern every
call (decode plan built per call)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd  # noqa: E402

k, r, S = 4096, 1024, 1024
rng = np.random.default_rng(1)
syms = [np.zeros(S, np.uint8) for _ in range(k + r)]
for i in range(k):
    syms[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
rs = rs_amd.RS()
inf, rep = syms[:k], syms[k:]


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


enc_ms = timed(lambda: rs.generate_repair_symbols(inf, rep), 5)
keep = [s.copy() for s in syms]
fixed = np.zeros(k + r, bool)
fixed[rng.choice(k + r, r, replace=False)] = True


def reset(pattern):  # the codeword back, the pattern's symbols erased (untimed)
    for i in range(k + r):
        syms[i][:] = keep[i]
    for i in np.nonzero(pattern)[0]:
        syms[i][:] = 0


def timed_dec(patterns):
    ts = []
    for p in patterns:
        reset(p)
        t0 = time.perf_counter()
        rs.restore_symbols(k, r, syms, p, int(p.sum()))
        ts.append(time.perf_counter() - t0)
        assert all(np.array_equal(syms[i], keep[i]) for i in range(k)), "not restored"
    return float(np.median(ts)) * 1e3


same_ms = timed_dec([fixed] * 5)
pats = []
for _ in range(6):
    p = np.zeros(k + r, bool)
    p[rng.choice(k + r, r, replace=False)] = True
    pats.append(p)
new_ms = timed_dec(pats)
print(json.dumps({"k": k, "r": r, "S": S, "encode_ms": round(enc_ms, 2), "decode_same_pattern_ms": round(same_ms, 2),
                  "decode_new_pattern_ms": round(new_ms, 2), "restored": True}))
