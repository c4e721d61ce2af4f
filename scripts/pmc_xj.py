"""One k=128 r=32 64 KiB configuration for PMC collection: n stripes, 3 encode launches (op enc) or
3 decode launches of the bench pattern (op dec), through the specialised kernels.
usage: pmc_xj.py <kernel: jit|v1jit> [n] [enc|dec]"""
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd
kind, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1024
op = sys.argv[3] if len(sys.argv) > 3 else "enc"
k, r, S = 128, 32, 65536
dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
rs_amd.fill_info(dev, k, 0x5EED)
c = rs_amd.Codec(k, r, jit=1, xj=1 if kind == "jit" else 0)
c.encode(dev)
er = rs_amd.bench_pattern(k, r)
for _ in range(3):
    if op == "enc":
        c.encode(dev)
    else:
        c.decode(dev, er)
torch.cuda.synchronize()
print(op, c.last_kernel, rs_amd.version())
c.close()
