#!/bin/bash
# Closing parity fuzz over every family with the final library (xj, generic, m16, route, reenc, batch,
# batch16, dropin, ps16, orbit, dropin_reg), then the smoke.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -u scripts/fuzz_parity.py 3051 360 > gpurun_out/fz_all.jsonl 2>&1 || { tail -5 gpurun_out/fz_all.jsonl; exit 1; }
tail -1 gpurun_out/fz_all.jsonl
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fz_smoke.log 2>&1 || { tail -5 gpurun_out/fz_smoke.log; exit 1; }
tail -1 gpurun_out/fz_smoke.log
