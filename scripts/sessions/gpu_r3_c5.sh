#!/bin/bash
# Round 3: C5 route tests, then the C5 bench line (decode: plain route + orbit k_bs16 for the bench pattern).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "c5 or m16 or max_n or golden_batch_api" > gpurun_out/r3_c5_tests.log 2>&1 || { tail -40 gpurun_out/r3_c5_tests.log; exit 1; }
tail -2 gpurun_out/r3_c5_tests.log
timeout -k 10 600 python -u bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 20 > gpurun_out/r3_bench_c5.log 2>&1 || { tail -5 gpurun_out/r3_bench_c5.log; exit 1; }
tail -1 gpurun_out/r3_bench_c5.log | cut -c1-1500
timeout -k 10 300 ./scripts/bench_hostops scripts/prev_lib/librs_amd_eaa4894.so > gpurun_out/r3_hostops_before.jsonl 2>&1 || { tail -5 gpurun_out/r3_hostops_before.jsonl; exit 1; }
timeout -k 10 300 ./scripts/bench_hostops reed-solomon_amd/librs_amd.so oracle/_ref/librs_ref.so > gpurun_out/r3_hostops.jsonl 2>&1 || { tail -5 gpurun_out/r3_hostops.jsonl; exit 1; }
cat gpurun_out/r3_hostops_before.jsonl gpurun_out/r3_hostops.jsonl
