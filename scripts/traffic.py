#!/usr/bin/env python3
"""HBM traffic per launch of the dominant kernel from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE in separate runs of `bench.py --profile-only`), corrected as MI355X_MICROARCH.md's HBM
section prescribes: FETCH_SIZE (KiB) reports half the bytes of wide streaming reads on gfx950, so
it is doubled; WRITE_SIZE (KiB) is taken as is.

usage: traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR CONFIG_KEY BENCH_KERNEL > traffic.json"""
import csv
import glob
import json
import os
import sys



def per_dispatch(d, counter, kern):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kern in row["Kernel_Name"] and row["Counter_Name"] == counter:
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kern} under {d}")
    return sorted(vals.values())


fd, wd, kern, cfg, bench_kernel = sys.argv[1:6]
# the bench line of the profiled run names the dominant kernel exactly (JIT kernels carry the hash of
# their generated source: "rs_xj[32x128:c80999d0]"), which identifies the measured code
for line in open(os.path.join(os.path.dirname(fd.rstrip("/")), "tr_fetch.log")):
    if line.startswith("{"):
        bench_kernel = json.loads(line)["roofline"]["kernel"]
fetch = per_dispatch(fd, "FETCH_SIZE", kern)
write = per_dispatch(wd, "WRITE_SIZE", kern)
med = lambda v: v[len(v) // 2]
fetch_b = med(fetch) * 1024 * 2
write_b = med(write) * 1024
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
from srchash import kernel_src_hash  # noqa: E402
print(json.dumps({"src_hash": kernel_src_hash(bench_kernel), "kernel": kern, "bench_kernel": bench_kernel, "config": cfg,
                  "fetch_bytes_corrected": fetch_b, "write_bytes": write_b, "traffic_bytes": fetch_b + write_b,
                  "dispatches": [len(fetch), len(write)],
                  "raw_kib": {"FETCH_SIZE": med(fetch), "WRITE_SIZE": med(write)}}, indent=1))
