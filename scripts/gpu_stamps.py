"""Phase timing of the production m8 kernel (mode 17 = k_apply_m8_lds<0> with s_memtime counters):
per wave, cycles spent in [batch prologue: DMA issue + ring reads + coordinate lookups],
[4 asm steps], [DMA wait + barrier], and in total; k=128 r=32 64 KiB, encode."""
import ctypes, json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
# ablation modes exist only in the diagnostic build (make -C reed-solomon_amd diag)
os.environ.setdefault("RS_AMD_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd", "librs_amd_diag.so"))
import rs_amd
k, r, S, n = 128, 32, 65536, int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
rs_amd.fill_info(dev, k, 0x5EED)
blocks = n * (S // 2048)
st = torch.zeros(blocks * 16, dtype=torch.int64, device="cuda")
res = {}
for mode in (2, 17):
    c = rs_amd.Codec(k, r, m8_mode=mode)
    if mode == 17:
        c.set_option("stamp_buffer", st.data_ptr())
    c.encode(dev); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); c.encode(dev); b.record(); torch.cuda.synchronize()
    res[f"ms_mode{mode}"] = round(a.elapsed_time(b), 3)
    c.close()
ph = st.view(blocks * 4, 4).cpu().numpy().astype(np.float64)
nb = k // 4
names = ["prologue_coords", "asm4", "wait_barrier", "total"]
res.update({f"{nm}_per_batch": round(float(ph[:, i].mean()) / nb, 1) for i, nm in enumerate(names)})
res["total_per_wave"] = round(float(ph[:, 3].mean()), 0)
res["p10_p90_total"] = [round(float(np.percentile(ph[:, 3], q)), 0) for q in (10, 90)]
print(json.dumps(res))
