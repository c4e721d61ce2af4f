#!/usr/bin/env python3
"""Summarise scripts/gpu_cs16t_stalls.sh: median SQ counters per k_cs16t dispatch of the C5 bench (encode
and decode launches alike: 1024 stripes of k=4096 r=1024 1 KiB), per wave and per group step.
usage: cs16t_stalls.py DIR [duration_ms]"""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/cs16t_stalls"
tot = {}
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for row in csv.DictReader(open(f)):
        if "k_cs16t" in row["Kernel_Name"]:
            vals[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    ids = sorted(vals, key=int)
    for c in (vals[ids[0]] if ids else {}):
        xs = sorted(vals[i][c] for i in ids)
        tot[c] = xs[len(xs) // 2]
waves = tot.get("SQ_WAVES", 1.0)
print("# k_cs16t at C5 (median over dispatches); counter: per dispatch | per wave")
for c in sorted(tot):
    print(f"{c:24s} {tot[c]:14.4g} | {tot[c] / waves:12.1f}")
