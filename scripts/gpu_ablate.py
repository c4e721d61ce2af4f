"""Timing ablation of the m8 asm kernel (one process, interleaved rounds): full, no index switching,
build only, lookups only. Results of the ablated variants are wrong by construction."""
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
# ablation modes exist only in the diagnostic build (make -C reed-solomon_amd diag)
os.environ.setdefault("RS_AMD_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd", "librs_amd_diag.so"))
import rs_amd
k, r, S, n = 128, 32, 65536, int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
rs_amd.fill_info(dev, k, 0x5EED)
modes = {"lds": 2, "reg4": 3, "lds_noidx": 10, "lds_build": 11, "lds_look": 12, "lds_nop": 13, "lds_split_mul": 14,
         "lds_plain": 15, "reg4_nop": 16, "v1": 18, "v1_plain": 19}
codecs = {m: rs_amd.Codec(k, r, m8_mode=v, jit=0) for m, v in modes.items()}
codecs["jit"] = rs_amd.Codec(k, r, jit=1)
res = {m: [] for m in codecs}
# bit-exactness of the schedules that must be correct, against the table kernel (mode 0)
ref = dev[:8].clone()
rs_amd.Codec(k, r, m8_mode=0, jit=0).encode(ref)
for m in ("lds", "reg4", "lds_split_mul", "v1", "jit"):
    d = dev[:8].clone()
    codecs[m].encode(d)
    torch.cuda.synchronize()
    print(json.dumps({"variant": m, "bitexact": bool(torch.equal(d, ref))}))
for rnd in range(4):
    for m, c in codecs.items():
        c.encode(dev); torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); c.encode(dev); b.record(); torch.cuda.synchronize()
        if rnd: res[m].append(a.elapsed_time(b))
for c in codecs.values():
    c.close()
for m, v in res.items():
    ms = float(np.median(v))
    print(json.dumps({"variant": m, "ms": round(ms, 3), "GBps": round(n * (k + r) * S / ms / 1e6, 1)}))
