#!/usr/bin/env python3
"""Summarise scripts/gpu_xj_phases.sh: per-launch SQ counters of the C3 XOR kernels with each timing
ablation, and the per-phase VALU per 256-byte column (full - ablated). usage: xj_phases.py DIR"""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/xj_phases"
COLS = 1024 * 65536 // 256  # scripts/pmc_xj.py: 1024 stripes of 64 KiB symbols, 256-byte columns
print("# C3 (k=128, r=32, 64 KiB) XOR kernels, 1024 stripes per launch = %d columns; median of the launches" % COLS)
print("# op ablation kernel | SQ_INSTS_VALU/column SQ_INSTS_SALU/column SQ_WAVES | kernel ms | GRBM_GUI_ACTIVE/8 / ms = MHz")
per = {}
for op in ("enc", "dec"):
    for ab in (0, 1, 2, 4):
        vals = collections.defaultdict(lambda: collections.defaultdict(float))
        name = {}
        for f in glob.glob(f"{d}/{op}_a{ab}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if row["Kernel_Name"].startswith("rs_xj"):
                    vals[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
                    name[row["Dispatch_Id"]] = row["Kernel_Name"].split("(")[0]
        dur = {}
        for f in glob.glob(f"{d}/{op}_a{ab}/**/*kernel_trace.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                dur[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
        ids = sorted(vals, key=int)[1:]  # the first launch of each run is the encode that fills the repair symbols
        if not ids:
            continue
        med = lambda xs: sorted(xs)[len(xs) // 2]
        valu = med([vals[i]["SQ_INSTS_VALU"] for i in ids]) / COLS
        salu = med([vals[i]["SQ_INSTS_SALU"] for i in ids]) / COLS
        ms = med([dur[i] for i in ids])
        mhz = med([vals[i]["GRBM_GUI_ACTIVE"] / 8 / (dur[i] * 1e3) for i in ids])
        per[(op, ab)] = valu
        print(f"{op} {ab} {name[ids[0]]} | {valu:.0f} {salu:.0f} {med([vals[i]['SQ_WAVES'] for i in ids]):.0f} | {ms:.3f} | {mhz:.0f}")
print("# per-phase VALU per column (full - ablated): finish = a0 - a1, rows = a0 - a2, tables = a0 - a4, rest")
for op in ("enc", "dec"):
    if (op, 0) not in per:
        continue
    f, r, t = per[(op, 0)] - per[(op, 1)], per[(op, 0)] - per[(op, 2)], per[(op, 0)] - per[(op, 4)]
    tot = per[(op, 0)]
    print(f"{op}: total {tot:.0f} = rows {r:.0f} ({100 * r / tot:.1f} %) + finish {f:.0f} ({100 * f / tot:.1f} %) + "
          f"tables {t:.0f} ({100 * t / tot:.1f} %) + loads/addressing/loop {tot - f - r - t:.0f}")
