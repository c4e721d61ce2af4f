#!/bin/bash
# Per-stripe C5 route with the overlapped syndrome stream: record-MiB (chunk size) sweep.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PS_REC_MIB=256,512,2048 timeout -k 10 400 python3 -u scripts/bench_patterns_c5.py 1024 > gpurun_out/ps_chunks.log 2>&1
rc=$?; cat gpurun_out/ps_chunks.log; exit $rc
