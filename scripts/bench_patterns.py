"""rsg_decode_batch with a different erasure pattern on every stripe (C3 shape): device-built plans
(batch_plans=1) against host plans per pattern (batch_plans=0), and the single-pattern decode of the
same stripes for reference. GB/s counts the algorithmic bytes of each stripe: survivors read
(k + r - t) + information symbols written (t_info)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd  # noqa: E402

k, r, S = 128, 32, 65536
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
mode = sys.argv[2] if len(sys.argv) > 2 else "t32info"
only = set(sys.argv[3].split(",")) if len(sys.argv) > 3 else None  # case labels to run (profiling)
rng = np.random.default_rng(5)
pats = np.zeros((n, k + r), bool)
for s in range(n):
    if mode == "t32info":  # r information erasures, a different set per stripe
        pats[s, rng.choice(k, r, replace=False)] = True
    else:  # 1..r erasures anywhere
        pats[s, rng.choice(k + r, int(rng.integers(1, r + 1)), replace=False)] = True
t = pats.sum(1)
tinfo = pats[:, :k].sum(1)
alg = float(((k + r - t) + tinfo)[tinfo > 0].sum()) * S
dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
rs_amd.fill_info(dev, k, seed=0x5EED)
enc = rs_amd.Codec(k, r)
enc.encode(dev)
torch.cuda.synchronize()


def fp():
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    rs_amd.fingerprint(dev, 0, k, out)
    return out


ref_fp = fp()
mask = torch.from_numpy(pats).to("cuda")


def run(codec, label, reps):
    if only is not None and label not in only:
        return
    times, host = [], []
    for _ in range(reps):
        dev.masked_fill_(mask[:, :, None], 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        codec.decode_batch(dev, pats)
        host.append(time.perf_counter() - t0)  # the call returns once every launch is queued
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    ok = bool(torch.equal(fp(), ref_fp))
    ms = float(np.median(times)) * 1e3
    print(json.dumps({"case": label, "stripes": n, "patterns": mode, "ms": round(ms, 3),
                      "GBps": round(alg / ms / 1e6, 1), "host_ms": round(float(np.median(host)) * 1e3, 3),
                      "restored": ok, "kernel": codec.last_kernel}), flush=True)


syn = rs_amd.Codec(k, r, batch_plans=1)
if os.environ.get("RS_PS8_OVERLAP"):  # A/B of the overlapped chunks (option m8_syn_overlap)
    syn.set_option("m8_syn_overlap", int(os.environ["RS_PS8_OVERLAP"]))
if os.environ.get("RS_PS8_ROUTE"):  # A/B of the fixed pass (option syn_route: 1 syndromes, 2 re-encode)
    syn.set_option("syn_route", int(os.environ["RS_PS8_ROUTE"]))
if os.environ.get("RS_PS8_KERNEL"):  # A/B of the per-stripe solve kernel (option m8_ps_kernel)
    syn.set_option("m8_ps_kernel", int(os.environ["RS_PS8_KERNEL"]))
if os.environ.get("RS_PS8_MASKED"):  # A/B of the masked fixed pass (option m8_syn_masked)
    syn.set_option("m8_syn_masked", int(os.environ["RS_PS8_MASKED"]))
if os.environ.get("RS_PS8_COORD"):  # A/B of the coordinate-output fixed pass (option m8_syn_coord)
    syn.set_option("m8_syn_coord", int(os.environ["RS_PS8_COORD"]))
if os.environ.get("RS_PS8_SCRATCH"):  # A/B of the fixed-pass scratch per chunk (option m8_syn_scratch_mib)
    syn.set_option("m8_syn_scratch_mib", int(os.environ["RS_PS8_SCRATCH"]))
if os.environ.get("RS_PS8_ABLATE"):  # timing ablations of the solve (diagnostic library, option m8_ps_ablate)
    syn.set_option("m8_ps_ablate", int(os.environ["RS_PS8_ABLATE"]))
if os.environ.get("RS_PS8_CPB"):  # A/B of column chunks per workgroup of that kernel (option m8_ps_cpb)
    syn.set_option("m8_ps_cpb", int(os.environ["RS_PS8_CPB"]))
run(syn, "device_plans_syndrome", 5)
sur = rs_amd.Codec(k, r, batch_plans=1)
sur.set_option("syn_route", 0)
run(sur, "device_plans_survivor", 5)
if only is None or "host_plans" in only:
    run(rs_amd.Codec(k, r, batch_plans=0), "host_plans", 2)
# the same bytes with one shared pattern (t = r information erasures): generic and specialised kernels
one = np.zeros(k + r, bool)
one[np.arange(r) * (k // r)] = True
gen_kw = dict(jit=0, m8_mode=int(os.environ.get("RS_PS8_M8MODE", "18")))  # A/B of the generic V = 1 step
for label, kw in (("one_pattern_generic", gen_kw), ("one_pattern_xj", dict())):
    if only is not None and label not in only:
        continue
    c = rs_amd.Codec(k, r, **kw)
    times = []
    for _ in range(4):
        t0 = time.perf_counter()
        c.decode(dev, one)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    ms = float(np.median(times[1:])) * 1e3
    print(json.dumps({"case": label, "stripes": n, "ms": round(ms, 3),
                      "GBps": round(n * (k + r) * S / ms / 1e6, 1), "kernel": c.last_kernel}), flush=True)
