#!/bin/bash
# Round 3: per-stripe GF(2^16) route -- its GPU tests, the full suite, then the C5 pattern bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "per_stripe_route or m16_stream_plans or c5_bench_decode or two_streams" > gpurun_out/r3_ps16_tests.log 2>&1 || { tail -40 gpurun_out/r3_ps16_tests.log; exit 1; }
tail -3 gpurun_out/r3_ps16_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gputest2.log 2>&1 || { tail -30 gpurun_out/r3_gputest2.log; exit 1; }
tail -1 gpurun_out/r3_gputest2.log
PS_REC_MIB=160,400 timeout -k 10 300 python -u scripts/bench_patterns_c5.py 256 > gpurun_out/r3_patterns_c5.log 2>&1 || { tail -10 gpurun_out/r3_patterns_c5.log; exit 1; }
cat gpurun_out/r3_patterns_c5.log
