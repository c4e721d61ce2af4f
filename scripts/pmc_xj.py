"""One k=128 r=32 64 KiB encode configuration for PMC collection (n stripes, 3 launches).
usage: pmc_xj.py <kernel: jit|v1jit> [n]"""
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd
kind, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1024
k, r, S = 128, 32, 65536
dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
rs_amd.fill_info(dev, k, 0x5EED)
c = rs_amd.Codec(k, r, jit=1, xj=1 if kind == "jit" else 0)
for _ in range(3):
    c.encode(dev)
torch.cuda.synchronize()
print(c.last_kernel)
c.close()
