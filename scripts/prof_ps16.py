"""The C5 per-stripe syndrome route alone (k=4096, r=1024, 1 KiB symbols, a random pattern of r erasures
per stripe), run three times, for a rocprofv3 kernel-trace breakdown of its kernels. Checks the restored
information against a fingerprint taken before the erasures."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd  # noqa: E402

k, r, S = 4096, 1024, 1024
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
rng = np.random.default_rng(7)
pats = np.zeros((n, k + r), bool)
for s in range(n):
    pats[s, rng.choice(k + r, r, replace=False)] = True
dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
rs_amd.fill_info(dev, k, seed=0x5EED)
codec = rs_amd.Codec(k, r)
codec.encode(dev)
out = torch.empty(n, dtype=torch.int64, device="cuda")
rs_amd.fingerprint(dev, 0, k, out)
ref = out.clone()
mask = torch.from_numpy(pats).to("cuda")
for it in range(3):
    dev.masked_fill_(mask[:, :, None], 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    codec.decode_batch(dev, pats)
    torch.cuda.synchronize()
    print(f"run {it}: {1e3 * (time.perf_counter() - t0):.2f} ms {codec.last_kernel}", flush=True)
rs_amd.fingerprint(dev, 0, k, out)
assert torch.equal(out, ref), "per-stripe decode did not restore the information"
print("restored", flush=True)
