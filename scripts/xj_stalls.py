#!/usr/bin/env python3
"""Summarise scripts/gpu_xj_stalls.sh: median per-launch SQ counters of the rs_xj encode kernel (first
launch dropped), per wave and per 256-byte column. usage: xj_stalls.py DIR"""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/xj_stalls"
COLS = 1024 * 65536 // 256
tot = {}
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for row in csv.DictReader(open(f)):
        if row["Kernel_Name"].startswith("rs_xj"):
            vals[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    ids = sorted(vals, key=int)[1:]
    for c in (vals[ids[0]] if ids else {}):
        xs = sorted(vals[i][c] for i in ids)
        tot[c] = xs[len(xs) // 2]
waves = tot.get("SQ_WAVES", 2 * COLS)
print("# rs_xj encode, 1024 C3 stripes per launch (%d columns); counter: per launch | per wave | per column" % COLS)
for c in sorted(tot):
    print(f"{c:24s} {tot[c]:14.4g} | {tot[c] / waves:10.1f} | {tot[c] / COLS:10.1f}")
