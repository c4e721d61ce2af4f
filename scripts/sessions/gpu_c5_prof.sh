#!/bin/bash
# rocprofv3 kernel statistics of the C5 syndrome route (k_cs16 vs the second stage).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o run -- python3 bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 3 --warmup 1 --no-cpu --profile-only > gpurun_out/c5prof/bench.log 2>&1
find gpurun_out/c5prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/c5prof/kernel_stats.csv \;
