#!/bin/bash
# Round-3 line for every single-GPU config with its CPU baseline: C2 (k=10 r=4 4 KiB, 1024 stripes and a
# large batch), C5 (k=4096 r=1024 1 KiB, 1024 stripes), C3 at 20 steps.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --k 10 --r 4 --symbol 4096 --stripes 1024 --steps 200 > gpurun_out/cf_c2_1024.log 2>&1 || { tail -5 gpurun_out/cf_c2_1024.log; exit 1; }
tail -1 gpurun_out/cf_c2_1024.log | cut -c1-200
timeout -k 10 300 python bench.py --k 10 --r 4 --symbol 4096 --stripes 262144 --steps 50 > gpurun_out/cf_c2_big.log 2>&1 || { tail -5 gpurun_out/cf_c2_big.log; exit 1; }
tail -1 gpurun_out/cf_c2_big.log | cut -c1-200
timeout -k 10 400 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 20 > gpurun_out/cf_c5.log 2>&1 || { tail -5 gpurun_out/cf_c5.log; exit 1; }
tail -1 gpurun_out/cf_c5.log | cut -c1-200
