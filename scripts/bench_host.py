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
for _ in range(3):  # warm: decode plan, its specialised kernel from the third call (cached on disk)
    assert rs.restore_symbols(k, r, stripes[0], er, t) == 0
    for i in np.nonzero(er)[0]:
        stripes[0][i][:] = 0
t0 = time.perf_counter()
for s in stripes:
    assert rs.restore_symbols(k, r, s, er, t) == 0
t_dec = time.perf_counter() - t0
assert all(np.array_equal(a, b) for s, kp in zip(stripes, keep) for a, b in zip(s[:k], kp))
rs.close()
out["dropin_encode_GBps"] = round(n_a * (k + r) * S / t_enc / 1e9, 2)
out["dropin_decode_GBps"] = round(n_a * (k + t) * S / t_dec / 1e9, 2)
out["dropin_stripes"] = n_a

# (b) batched pinned pipeline: info [n][k][S] and repair [n][r][S] in pinned host memory, device
# chunks with separate contiguous info / repair buffers (rsg_encode takes both layouts), so every
# copy is one contiguous DMA
n_b, chunk = 256, 16
h_info = torch.from_numpy(rng.integers(0, 256, (n_b, k, S), dtype=np.uint8)).pin_memory()
h_rep = torch.empty((n_b, r, S), dtype=torch.uint8).pin_memory()
codec = rs_amd.Codec(k, r)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
d_info = [torch.empty((chunk, k, S), dtype=torch.uint8, device="cuda") for _ in range(2)]
d_rep = [torch.empty((chunk, r, S), dtype=torch.uint8, device="cuda") for _ in range(2)]
d_full = [torch.empty((chunk, k + r, S), dtype=torch.uint8, device="cuda") for _ in range(2)]
h_full = torch.empty((n_b, k + r, S), dtype=torch.uint8).pin_memory()


def enc_pipeline():
    for c0 in range(0, n_b, chunk):
        j = (c0 // chunk) % 2
        st = streams[j]
        with torch.cuda.stream(st):
            d_info[j].copy_(h_info[c0:c0 + chunk], non_blocking=True)
            rc = codec.encode_raw(d_info[j].data_ptr(), k * S, S, d_rep[j].data_ptr(), r * S, S, chunk, S, st)
            assert rc == 0
            h_rep[c0:c0 + chunk].copy_(d_rep[j], non_blocking=True)
    torch.cuda.synchronize()


def dec_pipeline():
    for c0 in range(0, n_b, chunk):
        j = (c0 // chunk) % 2
        st = streams[j]
        with torch.cuda.stream(st):
            d_full[j].copy_(h_full[c0:c0 + chunk], non_blocking=True)
            codec.decode(d_full[j], er, stream=st)
            for s in range(chunk):  # restored information symbols back: contiguous k*S per stripe
                h_full[c0 + s, :k].copy_(d_full[j][s, :k], non_blocking=True)
    torch.cuda.synchronize()


enc_pipeline()
t0 = time.perf_counter()
enc_pipeline()
t_enc = time.perf_counter() - t0
h_full[:, :k] = h_info
h_full[:, k:] = h_rep
h_full[:, torch.from_numpy(np.nonzero(er)[0])] = 0
dec_pipeline()
t0 = time.perf_counter()
dec_pipeline()
t_dec = time.perf_counter() - t0
assert torch.equal(h_full[:, :k], h_info)
out["pipeline_encode_GBps"] = round(n_b * (k + r) * S / t_enc / 1e9, 2)
out["pipeline_decode_GBps"] = round(n_b * (k + t) * S / t_dec / 1e9, 2)
out["pipeline"] = (f"{n_b} stripes, {chunk}-stripe chunks, 2 streams; encode copies k symbols in and r out, "
                   f"decode copies the whole stripe in and the k information symbols out")

# (d) the library's own host-memory batch API (rsg_encode_host / rsg_decode_host) on pinned stripes
h_all = torch.zeros((n_b, k + r, S), dtype=torch.uint8).pin_memory()
h_all[:, :k] = h_info
codec.encode_host(h_all)  # warm (device batch buffers, streams)
t0 = time.perf_counter()
codec.encode_host(h_all)
t_enc = time.perf_counter() - t0
assert torch.equal(h_all[:, k:], h_rep)
h_all[:, torch.from_numpy(np.nonzero(er)[0])] = 0
codec.decode_host(h_all, er)
h_all[:, torch.from_numpy(np.nonzero(er)[0])] = 0
t0 = time.perf_counter()
codec.decode_host(h_all, er)
t_dec = time.perf_counter() - t0
assert torch.equal(h_all[:, :k], h_info)
out["host_api_encode_GBps"] = round(n_b * (k + r) * S / t_enc / 1e9, 2)
out["host_api_decode_GBps"] = round(n_b * (k + t) * S / t_dec / 1e9, 2)
out["host_api"] = (f"rsg_encode_host / rsg_decode_host, {n_b} pinned stripes: encode copies k symbols in and r "
                   f"out, decode copies the surviving symbols in and only the t restored symbols out")
print(json.dumps(out))
