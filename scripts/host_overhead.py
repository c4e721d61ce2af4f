"""Host time per batched API call at C2 shapes (k=10, r=4, 4 KiB): wall time of N back-to-back calls
on tiny grids (the GPU work per call is a few microseconds, so the loop runs at the host's pace), and the
same for torch event records and an empty torch kernel for scale. usage: host_overhead.py [N]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
k, r, S = 10, 4, 4096
dev = torch.zeros((1, k + r, S), dtype=torch.uint8, device="cuda")
c = rs_amd.Codec(k, r)
er = rs_amd.bench_pattern(k, r)
st = torch.cuda.current_stream()


def rate(fn):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(N):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / N * 1e6


ev = torch.cuda.Event()
x = torch.zeros(1, device="cuda")
res = {"encode_us": rate(lambda: c.encode(dev, stream=st)), "decode_us": rate(lambda: c.decode(dev, er, stream=st)),
       "event_record_us": rate(lambda: ev.record(st)), "torch_add_us": rate(lambda: x.add_(1)),
       "encode_kernel": c.last_kernel}
print(res)
