#!/usr/bin/env python3
"""Merges scripts/traffic.py outputs (gpurun_out/<run>/c*affic.json) into profiles/traffic.json, the table
bench.py's `measured_traffic` reads. A record is keyed by (leg, bench_kernel, config, src_hash); a new
measurement of the same key replaces the old one, other records are kept.
usage: traffic_merge.py FILE.json [FILE.json ...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(REPO, "profiles", "traffic.json")


def key(rec):
    return (rec.get("leg"), rec.get("bench_kernel"), rec.get("config"), rec.get("src_hash"))


def main(paths, table=TABLE):
    with open(table) as f:
        doc = json.load(f)
    recs = doc["records"]
    added = replaced = 0
    for p in paths:
        with open(p) as f:
            new = json.load(f)
        for rec in new.get("records", [new]):
            old = [i for i, r in enumerate(recs) if key(r) == key(rec)]
            for i in reversed(old):
                del recs[i]
            replaced += bool(old)
            added += not old
            recs.append(rec)
    with open(table, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"{table}: {added} added, {replaced} replaced, {len(recs)} records")


if __name__ == "__main__":
    main(sys.argv[1:])
