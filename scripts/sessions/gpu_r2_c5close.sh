#!/bin/bash
# After a route-kernel change: full GPU suite, route / reenc fuzz, C5 bench line (with its traffic record).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/cc_suite.log 2>&1 || { tail -30 gpurun_out/cc_suite.log; exit 1; }
tail -1 gpurun_out/cc_suite.log
timeout -k 10 300 python -u scripts/fuzz_parity.py 31337 180 route,reenc,m16,batch16 > gpurun_out/cc_fuzz.jsonl 2>&1 || { tail -3 gpurun_out/cc_fuzz.jsonl; exit 1; }
tail -1 gpurun_out/cc_fuzz.jsonl
timeout -k 10 600 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 40 > gpurun_out/cc_c5.log 2>&1 || { tail -5 gpurun_out/cc_c5.log; exit 1; }
tail -1 gpurun_out/cc_c5.log | cut -c1-200
