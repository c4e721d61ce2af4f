#!/usr/bin/env python3
"""C2 (k=10, r=4, 4 KiB, 1024 stripes) launch time of the XOR kernels against RS_XJ_CPB (columns per
workgroup; the diagnostic library reads the generation knobs): at this size a launch is ~18 us and each wave
holds a few hundred VALU of work, so the workgroup count (16 per stripe at one column each) may bound it.
HIP events per launch on the launch stream, median of 200; round trip checked with fingerprints.
usage: c2_cpb_sweep.py [cpb ...]  -> one JSON line per setting"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "reed-solomon_amd"))
import rs_amd  # noqa: E402

D = rs_amd.diag_module()
k, r, S, n = 10, 4, 4096, 1024
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream()
erased = rs_amd.bench_pattern(k, r)
for cpb in [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8, 16]:
    os.environ["RS_XJ_CPB"] = str(cpb)
    codec = D.Codec(k, r, device=0)
    buf = torch.empty((n, k + r, S), dtype=torch.uint8, device=dev)
    rs_amd.fill_info(buf, k, 0x5EED, stream=stream)
    fp0 = torch.zeros(n, dtype=torch.int64, device=dev)
    rs_amd.fingerprint(buf, 0, k, fp0, stream=stream)
    for _ in range(5):
        codec.encode(buf, stream=stream)
        codec.decode(buf, erased, stream=stream)
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(200)]
    for e in ev:
        e[0].record(stream)
        codec.encode(buf, stream=stream)
        e[1].record(stream)
        codec.decode(buf, erased, stream=stream)
        e[2].record(stream)
    torch.cuda.synchronize()
    enc = float(np.median([a.elapsed_time(b) for a, b, _ in ev])) * 1e3
    dec = float(np.median([b.elapsed_time(c) for _, b, c in ev])) * 1e3
    buf[:, torch.from_numpy(erased).to(dev)] = 0xA5
    codec.decode(buf, erased, stream=stream)
    fp1 = torch.zeros(n, dtype=torch.int64, device=dev)
    rs_amd.fingerprint(buf, 0, k, fp1, stream=stream)
    torch.cuda.synchronize()
    by = n * (k + r) * S
    print(json.dumps({"cpb": cpb, "encode_us": round(enc, 2), "decode_us": round(dec, 2),
                      "GBps": round(2 * by / ((enc + dec) / 1e6) / 1e9, 1), "kernel": codec.last_kernel,
                      "roundtrip": bool(torch.equal(fp0, fp1))}), flush=True)
    codec.close()
