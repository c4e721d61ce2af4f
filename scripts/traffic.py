#!/usr/bin/env python3
"""HBM traffic per launch of the bench's encode and decode kernels from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in separate runs of `bench.py --profile-only`), corrected as
MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE (KiB) reports half the bytes of wide
streaming reads on gfx950, so it is doubled; WRITE_SIZE (KiB) is taken as is.

Records are keyed per launch by the exact kernel the bench line names for each leg
(config.kernel.encode / .decode): the specialised XOR kernels carry the hash of their generated source
in their symbol (rocprof "rs_xj_<hash>" = bench "rs_xj[RxK:<hash>]"), so the encode and decode kernels of
one run are told apart; compiled kernels are matched by name substring and source hash. A composite leg
(the GF(2^16) route: "cs16+bs16", ...) is the sum of its component kernels per launch, attributed by
dispatch order.

usage: traffic.py FETCH_DIR WRITE_DIR CONFIG_KEY > traffic.json"""
import csv
import glob
import json
import os
import re
import sys
import time


def per_dispatch(d, counter, match):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if match(row["Kernel_Name"]) and row["Counter_Name"] == counter:
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return sorted(vals.values())


# components of the composite GF(2^16) route legs (bench names "cs16t+bs16", "cs16t+bs16+xor+apply_m16_v1"; cs16 = the gpr-indexed syndrome kernel)
_PART = {"cs16": "rsamd::k_cs16(", "cs16t": "rsamd::k_cs16t(", "bs16": "rsamd::k_bs16(", "xor": "rsamd::k_xor_rows(",
         "apply_m16_v1": "k_apply_m16_v1<"}


def per_leg_composite(d, counter, legs):
    """Composite legs: every launch of a leg is a fixed sequence of component kernels. Walk the run's
    dispatches of those kernels in issue order, split them into the bench's legs (encode sequence,
    then decode sequence, per step) and return, per leg, the sorted per-occurrence sums."""
    parts = {p for seq in legs.values() for p in seq}
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            hit = [p for p in parts if _PART[p] in row["Kernel_Name"]]
            if hit:
                rows.append((int(row.get("Dispatch_Id") or row.get("Correlation_Id")), hit[0], float(row["Counter_Value"])))
    agg = {}
    for did, part, v in rows:  # counters may come per XCD / SE: sum per dispatch
        agg.setdefault(did, [part, 0.0])[1] += v
    seq = [agg[k] for k in sorted(agg)]
    order = ["encode", "decode"]
    out = {leg: [] for leg in legs}
    i, li = 0, 0
    while i < len(seq):
        leg = order[li % 2] if all(l in legs for l in order) else next(iter(legs))
        want = legs[leg]
        got = [p for p, _ in seq[i:i + len(want)]]
        if got != want:  # not at a leg boundary (e.g. a dense first launch): skip one dispatch
            i += 1
            continue
        split = {}
        for part, v in seq[i:i + len(want)]:
            split[part] = split.get(part, 0.0) + v
        out[leg].append((sum(v for _, v in seq[i:i + len(want)]), split))
        i += len(want)
        li += 1
    return {leg: sorted(v, key=lambda x: x[0]) for leg, v in out.items()}


def matcher(bench_kernel):
    m = re.match(r"rs_xj\[\d+x\d+:([0-9a-f]{8})\]$", bench_kernel)
    if m:
        sym = "rs_xj_" + m.group(1)
        return lambda name: name.split("(")[0].strip() == sym
    return lambda name: bench_kernel.split("[")[0] in name


def main():
    fd, wd, cfg = sys.argv[1:4]
    line = None
    for ln in open(fd.rstrip("/") + ".log"):  # the FETCH pass's bench output (its JSON line names the kernels)
        if ln.startswith("{"):
            line = json.loads(ln)
    if line is None:
        raise SystemExit(f"no bench line in {fd}.log")
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon_amd"))
    from srchash import kernel_src_hash
    med = lambda v: v[len(v) // 2]
    records = []
    kern = line["config"]["kernel"]
    legs = {leg: name.split("+") for leg, name in kern.items() if "+" in name}
    if legs:
        fetch_c = per_leg_composite(fd, "FETCH_SIZE", legs)
        write_c = per_leg_composite(wd, "WRITE_SIZE", legs)
    for leg, bench_kernel in sorted(kern.items()):
        if leg in legs:
            fetch, write = fetch_c[leg], write_c[leg]
            if not fetch or not write:
                print(f"no complete {bench_kernel} sequences", file=sys.stderr)
                continue
            (fv, fsplit), (wv, wsplit) = med(fetch), med(write)
            fetch_b = fv * 1024 * 2
            write_b = wv * 1024
            # per component kernel (of the median launch): corrected fetch + write bytes
            split = {part: {"fetch_bytes_corrected": fsplit.get(part, 0.0) * 1024 * 2,
                            "write_bytes": wsplit.get(part, 0.0) * 1024} for part in legs[leg]}
            records.append({"leg": leg, "src_hash": kernel_src_hash(bench_kernel), "bench_kernel": bench_kernel,
                            "config": cfg, "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
                            "traffic_bytes": fetch_b + write_b, "dispatches": [len(fetch), len(write)],
                            "components": legs[leg], "component_bytes": split,
                            "raw_kib": {"FETCH_SIZE": fv, "WRITE_SIZE": wv}})
            continue
        match = matcher(bench_kernel)
        fetch = per_dispatch(fd, "FETCH_SIZE", match)
        write = per_dispatch(wd, "WRITE_SIZE", match)
        if not fetch or not write:
            print(f"no FETCH_SIZE / WRITE_SIZE rows for {bench_kernel}", file=sys.stderr)
            continue
        fetch_b = med(fetch) * 1024 * 2
        write_b = med(write) * 1024
        records.append({"leg": leg, "src_hash": kernel_src_hash(bench_kernel), "bench_kernel": bench_kernel,
                        "config": cfg, "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
                        "traffic_bytes": fetch_b + write_b, "dispatches": [len(fetch), len(write)],
                        "raw_kib": {"FETCH_SIZE": med(fetch), "WRITE_SIZE": med(write)}})
    if not records:
        raise SystemExit("no records")
    stamp = time.strftime("%Y-%m-%d")
    for rec in records:
        rec["measured"] = stamp
    print(json.dumps({"records": records}, indent=1))


if __name__ == "__main__":
    main()
