#!/bin/bash
# Round 3: kernel times of the per-stripe GF(2^16) route at C5 (256 all-distinct t = 1024 patterns).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ps16prof -o run -- python3 scripts/bench_patterns_c5.py 256 > gpurun_out/r3_ps16_prof.log 2>&1 || { tail -20 gpurun_out/r3_ps16_prof.log; exit 1; }
cat gpurun_out/r3_ps16_prof.log | grep case
f=$(find gpurun_out/ps16prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r3_ps16_kernel_stats.csv; cut -d, -f1-8 gpurun_out/r3_ps16_kernel_stats.csv | head -20
