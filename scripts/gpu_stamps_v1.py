"""Phase stamps of the V = 1 GF(256) kernel (diagnostic library, RS_AMD_LIB=.../librs_amd_diag.so): the
per-stripe solve of rsg_decode_batch (m8_ps_kernel 7; 4096 C3 stripes, all-distinct t = 32 information
erasures, re-encode route) against one shared pattern on the generic kernel (m8_mode 21; 512 stripes,
K = 128). Per wave, s_memtime cycles of table setup, ring prologue, input steps, DMA waits + barriers and
the output stage (rs_device.h m8_v1_run STAMP); prints the means per wave and per input.
TEST INFRASTRUCTURE: timing only."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd  # noqa: E402

k, r, S = 128, 32, 65536
NAMES = ["setup", "prologue", "steps", "waits", "outputs", "total"]


def summary(label, st, K):
    a = st.view(-1, 8).cpu().numpy().astype(np.int64)
    a = a[a[:, 5] > 0]
    m = a[:, :6].mean(0)
    row = {"case": label, "waves": int(a.shape[0]), "K": K}
    row.update({n: round(float(v)) for n, v in zip(NAMES, m)})
    row["steps_per_input"] = round(float(m[2]) / K, 1)
    span = (a[:, 7].max() - a[:, 6].min())
    row["busy_waves_avg"] = round(float(a[:, 5].sum()) / float(span), 1) if span > 0 else None
    print(json.dumps(row), flush=True)


rng = np.random.default_rng(5)
n = 4096
pats = np.zeros((n, k + r), bool)
for s in range(n):
    pats[s, rng.choice(k, r, replace=False)] = True
dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
rs_amd.fill_info(dev, k, seed=0x5EED)
rs_amd.Codec(k, r).encode(dev)
st = torch.zeros(8 << 20, dtype=torch.int64, device="cuda")
c = rs_amd.Codec(k, r, batch_plans=1)
c.set_option("m8_ps_kernel", 7)
c.set_option("stamp_buffer", st.data_ptr())
for _ in range(2):
    st.zero_()
    c.decode_batch(dev, pats)
    torch.cuda.synchronize()
summary("per_stripe_t32", st, 32)

one = np.zeros(k + r, bool)
one[np.arange(r) * (k // r)] = True
g = rs_amd.Codec(k, r, jit=0, m8_mode=21)
g.set_option("stamp_buffer", st.data_ptr())
sub = dev[:512]
for _ in range(2):
    st.zero_()
    g.decode(sub, one)
    torch.cuda.synchronize()
summary("one_pattern_k128", st, 128)
