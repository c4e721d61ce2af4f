#!/bin/bash
# C5 (k=4096, r=1024, 1 KiB symbols, 1024 stripes): syndrome route vs the dense GF(2^16) kernel, and
# the GPU tests of the m = 16 paths.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "m16 or c5 or wide or large_n or max_n or symbol_ops or surface" > gpurun_out/r2_c5_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 5 --warmup 2 --no-cpu > gpurun_out/r2_c5_route.log 2>&1 &&
timeout -k 10 300 python -u bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 5 --warmup 2 --no-cpu --opt m16_route=0 > gpurun_out/r2_c5_dense.log 2>&1
