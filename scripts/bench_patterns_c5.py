"""rsg_decode_batch at C5 (k=4096, r=1024, 1 KiB symbols) with a different erasure pattern on every
stripe: GF(2^16) codes take the per-stripe syndrome route (default since round 3: one syndrome pass over every
stripe, a device-built t_info x t solve per stripe) or, with m16_ps=0, build one decode plan per
pattern on the device and launch per pattern (one plan rebuilt on the stream per pattern), or cache
per-pattern plans (batch_plans=0). Compared with one shared pattern over the same stripes.
m16_ps=2 is the re-encode variant (the codec's encode route over the information slots, + the received repair
rows, then a t_info x t_info Cauchy solve per stripe). GB/s counts survivors read + information symbols written."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
import rs_amd  # noqa: E402

k, r, S = 4096, 1024, 1024
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rng = np.random.default_rng(7)
pats = np.zeros((n, k + r), bool)
tpat = int(os.environ.get("RS_C5_T", r))  # erasures per stripe (default t = r), anywhere
for s in range(n):
    pats[s, rng.choice(k + r, tpat, replace=False)] = True
t = pats.sum(1)
tinfo = pats[:, :k].sum(1)
alg = float(((k + r - t) + tinfo).sum()) * S
dev = torch.empty((n, k + r, S), dtype=torch.uint8, device="cuda")
rs_amd.fill_info(dev, k, seed=0x5EED)
codec = rs_amd.Codec(k, r)
codec.set_option("m16_ps", 1)  # the syndrome route (the default, 3, picks by the batch's largest pattern)
codec.encode(dev)
torch.cuda.synchronize()


def fp():
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    rs_amd.fingerprint(dev, 0, k, out)
    return out


ref_fp = fp()
orig = dev.clone()  # the codewords: erased repair slots stay zero after a decode (only info is restored)
mask = torch.from_numpy(pats).to("cuda")
old = rs_amd.Codec(k, r)
old.set_option("m16_ps", 0)
serial = rs_amd.Codec(k, r)
serial.set_option("m16_ps", 1)
serial.set_option("m16_ps_overlap", 0)
reenc = rs_amd.Codec(k, r)
reenc.set_option("m16_ps", 2)  # the re-encode variant: encode route over the information slots + W' per stripe
runs = [("distinct_patterns_ps16_route", codec), ("distinct_patterns_ps16_reenc", reenc),
        ("distinct_patterns_ps16_route_no_overlap", serial)]
for mib in [int(x) for x in os.environ.get("PS_REC_MIB", "").split(",") if x]:  # chunk-size sweep
    cm = rs_amd.Codec(k, r)
    cm.set_option("m16_ps_rec_mib", mib)
    runs.append((f"distinct_patterns_ps16_route_rec{mib}MiB", cm))
if not os.environ.get("RS_C5_ROUTES_ONLY"):
    runs += [("distinct_patterns_stream_plans", old), ("distinct_patterns_cached_plans", rs_amd.Codec(k, r, batch_plans=0))]
for label, cdc in runs:
    times = []
    for _ in range(3):
        dev.masked_fill_(mask[:, :, None], 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cdc.decode_batch(dev, pats)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    ok = bool(torch.equal(fp(), ref_fp))
    ms = float(np.median(times)) * 1e3
    print(json.dumps({"case": label, "k": k, "r": r, "S": S, "stripes": n, "ms": round(ms, 3),
                      "ms_per_stripe": round(ms / n, 3), "GBps": round(alg / ms / 1e6, 2), "restored": ok,
                      "kernel": cdc.last_kernel}), flush=True)
one = pats[0]
dev.copy_(orig)
dev.masked_fill_(torch.from_numpy(one).to("cuda")[None, :, None], 0)
times = []
for _ in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    codec.decode(dev, one)
    torch.cuda.synchronize()
    times.append(time.perf_counter() - t0)
ok = bool(torch.equal(fp(), ref_fp))
ms = float(np.median(times[1:])) * 1e3
alg1 = float(n * ((k + r - one.sum()) + one[:k].sum())) * S
print(json.dumps({"case": "one_pattern", "stripes": n, "ms": round(ms, 3), "ms_per_stripe": round(ms / n, 3),
                  "GBps": round(alg1 / ms / 1e6, 2), "restored": ok, "kernel": codec.last_kernel}), flush=True)
