#!/usr/bin/env python3
"""PCIe-inclusive (host-memory) rates for DESIGN.md -- never bench.py's `value`.

(a) drop-in API: the reference-compatible per-call rs_generate_repair_symbols / rs_restore_symbols on
    host symbols (one stripe per call: gather into pinned staging, H2D, kernel, D2H, scatter);
(b) batched pipeline: stripes in pinned host memory, chunks double-buffered over two HIP streams
    (H2D info -> encode -> D2H repair; H2D stripe -> decode -> D2H restored);
(c) raw pinned H2D / D2H copy bandwidth (the ceiling for (b)).
Configuration C3: k=128, r=32, 64 KiB symbols; decode t = 32 information erasures at i*4."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd  # noqa: E402

k, r, S = 128, 32, 65536
er = rs_amd.bench_pattern(k, r)
t = int(er.sum())
out = {}

# (c) raw copies
host = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
dev = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
for name, (dst, src) in {"h2d": (dev, host), "d2h": (host, dev)}.items():
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    out[f"pcie_{name}_GBps"] = round(5 * (1 << 30) / (time.perf_counter() - t0) / 1e9, 2)
del host, dev

# (a) drop-in API, one stripe per call
rs = rs_amd.RS()
n_a = 24
rng = np.random.default_rng(1)
stripes = [[rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k + r)] for _ in range(n_a)]
assert rs.generate_repair_symbols(stripes[0][:k], stripes[0][k:]) == 0  # warm (context, plans)
t0 = time.perf_counter()
for s in stripes:
    assert rs.generate_repair_symbols(s[:k], s[k:]) == 0
t_enc = time.perf_counter() - t0
keep = [[x.copy() for x in s[:k]] for s in stripes]
for s in stripes:
    for i in np.nonzero(er)[0]:
        s[i][:] = 0
t0 = time.perf_counter()
for s in stripes:
    assert rs.restore_symbols(k, r, s, er, t) == 0
t_dec = time.perf_counter() - t0
assert all(np.array_equal(a, b) for s, kp in zip(stripes, keep) for a, b in zip(s[:k], kp))
rs.close()
out["dropin_encode_GBps"] = round(n_a * (k + r) * S / t_enc / 1e9, 2)
out["dropin_decode_GBps"] = round(n_a * (k + t) * S / t_dec / 1e9, 2)
out["dropin_stripes"] = n_a

# (b) batched pinned pipeline
n_b, chunk = 192, 16
hst = torch.empty((n_b, k + r, S), dtype=torch.uint8).pin_memory()
hst[:, :k] = torch.from_numpy(rng.integers(0, 256, (k, S), dtype=np.uint8))[None]
codec = rs_amd.Codec(k, r)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
bufs = [torch.empty((chunk, k + r, S), dtype=torch.uint8, device="cuda") for _ in range(2)]
er_idx = torch.from_numpy(np.nonzero(er)[0])


def pipeline(decode):
    for c0 in range(0, n_b, chunk):
        j = (c0 // chunk) % 2
        st, b = streams[j], bufs[j]
        with torch.cuda.stream(st):
            if decode:
                b.copy_(hst[c0:c0 + chunk], non_blocking=True)
                codec.decode(b, er, stream=st)
                hst[c0:c0 + chunk, :k].copy_(b[:, :k], non_blocking=True)  # restored info (contiguous span)
            else:
                b[:, :k].copy_(hst[c0:c0 + chunk, :k], non_blocking=True)
                codec.encode(b, stream=st)
                hst[c0:c0 + chunk, k:].copy_(b[:, k:], non_blocking=True)
    torch.cuda.synchronize()


pipeline(False)
t0 = time.perf_counter()
pipeline(False)
t_enc = time.perf_counter() - t0
hst[:, er_idx] = 0
pipeline(True)
t0 = time.perf_counter()
pipeline(True)
t_dec = time.perf_counter() - t0
out["pipeline_encode_GBps"] = round(n_b * (k + r) * S / t_enc / 1e9, 2)
out["pipeline_decode_GBps"] = round(n_b * (k + t) * S / t_dec / 1e9, 2)
out["pipeline"] = f"{n_b} stripes, {chunk}-stripe chunks, 2 streams; decode copies the whole stripe in, k info symbols out"
print(json.dumps(out))
