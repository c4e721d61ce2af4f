#!/usr/bin/env python3
"""Per-dispatch means of every PMC counter under a rocprofv3 output tree, for kernels matching a
substring. usage: pmc_summary.py DIR KERNEL_SUBSTR"""
import csv, glob, sys
from collections import defaultdict
d, kern = sys.argv[1], sys.argv[2]
vals = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if kern in row["Kernel_Name"]:
            vals[row["Counter_Name"]][row.get("Dispatch_Id") or row.get("Correlation_Id")] += float(row["Counter_Value"])
for c in sorted(vals):
    v = list(vals[c].values())
    print(f"  {c:28s} {sum(v) / len(v):.4g}   ({len(v)} dispatches)")
