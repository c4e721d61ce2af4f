#!/bin/bash
# k_cs16t A/B on one box: this tree's library vs RS_AMD_LIB=scripts/prev_lib/<lib> (C5 bench, alternating),
# then the route tests on this tree's library.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PREV=scripts/prev_lib/${1:-librs_amd_r2tail.so}
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "cs16_threaded or c5_bench_decode or per_stripe_route or reenc or route or golden_batch_api" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 20 --no-cpu > gpurun_out/ab_new_$i.log 2>&1 || { tail -5 gpurun_out/ab_new_$i.log; exit 1; }
echo "new $i $(grep -o '"value": [0-9.]*' gpurun_out/ab_new_$i.log | head -1) $(grep -o '"encode_ms": [0-9.]*' gpurun_out/ab_new_$i.log) $(grep -o '"decode_ms": [0-9.]*' gpurun_out/ab_new_$i.log)"
RS_AMD_LIB=$PREV timeout -k 10 300 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 20 --no-cpu > gpurun_out/ab_prev_$i.log 2>&1 || { tail -5 gpurun_out/ab_prev_$i.log; exit 1; }
echo "prev $i $(grep -o '"value": [0-9.]*' gpurun_out/ab_prev_$i.log | head -1) $(grep -o '"encode_ms": [0-9.]*' gpurun_out/ab_prev_$i.log) $(grep -o '"decode_ms": [0-9.]*' gpurun_out/ab_prev_$i.log)"
done
