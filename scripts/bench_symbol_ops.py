#!/usr/bin/env python3
"""rsg_symbol_ops per-op cost over batch shapes (targets x ops per target x symbol size): HIP events around the
op-list copy + kernel with the stream held by a spin kernel while the call is queued (median of 5), the C
call's host time, and a numpy check of one target. RS_AMD_SYMOP_DW=1|2|4 picks the kernel's dwords per lane
(the library reads it once per process). One JSON line per shape."""
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
from _util import gf_tables  # noqa: E402

exp, log = gf_tables()
rng = np.random.default_rng(7)
stream = torch.cuda.current_stream()
shapes = [(1024, 128, 32), (1024, 1024, 4), (4096, 128, 32), (65536, 32, 32), (65536, 8, 128), (65536, 256, 8),
          (1 << 20, 8, 32)]
for S, n_t, per_t in shapes:
    src = torch.from_numpy(rng.integers(0, 256, (per_t, S), dtype=np.uint8)).cuda()
    tgt = torch.zeros((n_t, S), dtype=torch.uint8, device="cuda")
    coefs = rng.integers(2, 65536, (n_t, per_t))
    ops = np.zeros(n_t * per_t, rs_amd.SYMBOL_OP_DTYPE)
    ops["op"] = rs_amd.OP_MADD
    ops["a"] = tgt.data_ptr() + np.repeat(np.arange(n_t, dtype=np.uint64), per_t) * S
    ops["b"] = src.data_ptr() + np.tile(np.arange(per_t, dtype=np.uint64), n_t) * S
    ops["coef"] = coefs.reshape(-1)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(9)]
    host = []
    for e0, e1 in ev:
        tgt.zero_()
        torch.cuda.synchronize()
        torch.cuda._sleep(2_000_000)
        e0.record(stream)
        t0 = time.perf_counter()
        rs_amd.symbol_ops(ops, S, stream=stream)
        host.append(time.perf_counter() - t0)
        e1.record(stream)
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev[4:]]))  # the first calls fill the 4 staging slots
    got = tgt[0].cpu().numpy().view("<u2").astype(np.int64)
    ws = src.cpu().numpy().view("<u2").astype(np.int64)
    want = np.zeros_like(got)
    for j in range(per_t):
        want ^= np.where(ws[j] != 0, exp[(log[ws[j]] + log[coefs[0, j]]) % 65535], 0)
    n_ops = n_t * per_t
    print(json.dumps({"dw": os.environ.get("RS_AMD_SYMOP_DW", "default"), "S": S, "targets": n_t, "ops_per_target": per_t,
                      "call_ms": round(ms, 4), "us_per_op": round(ms * 1e3 / n_ops, 4),
                      "host_us_per_op": round(float(np.median(host[4:])) * 1e6 / n_ops, 4),
                      "source_GBps": round(n_ops * S / ms / 1e6, 1), "ok": bool(np.array_equal(got, want))}), flush=True)
