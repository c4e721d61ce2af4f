#!/usr/bin/env python3
"""Per-launch-shape statistics from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv): launches of one
kernel grouped by grid size, so the headline launches of a bench run (the full 8192-stripe grid) are told
apart from the same kernel's smaller launches in the extra legs (the host-memory pipeline runs the same
encode matrix, hence the same content-addressed rs_xj kernel, on 16-stripe batches).

usage: trace_split.py run_kernel_trace.csv [kernel-substring ...]  -> CSV on stdout:
kernel, grid, calls, average_ns, min_ns, max_ns"""
import csv
import sys


def split(path, names=()):
    groups = {}
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"]
        if names and not any(n in k for n in names):
            continue
        grid = f'{row["Grid_Size_X"]}x{row["Grid_Size_Y"]}x{row["Grid_Size_Z"]}'
        d = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        groups.setdefault((k, grid), []).append(d)
    return {key: (len(v), sum(v) / len(v), min(v), max(v)) for key, v in groups.items()}


def main(argv):
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "calls", "average_ns", "min_ns", "max_ns"])
    for (k, grid), (n, avg, lo, hi) in sorted(split(argv[1], argv[2:]).items(), key=lambda x: -x[1][0] * x[1][1]):
        w.writerow([k, grid, n, round(avg, 1), lo, hi])


if __name__ == "__main__":
    main(sys.argv)
