#!/bin/bash
# Full GPU suite, then the parity fuzz over every family (route / reenc with both block layouts).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/c2_suite.log 2>&1 || { tail -30 gpurun_out/c2_suite.log; exit 1; }
tail -1 gpurun_out/c2_suite.log
timeout -k 10 400 python -u scripts/fuzz_parity.py 4242 300 > gpurun_out/c2_fuzz.jsonl 2>&1 || { tail -5 gpurun_out/c2_fuzz.jsonl; exit 1; }
tail -2 gpurun_out/c2_fuzz.jsonl
