#!/bin/bash
# k_cs16t (threaded syndrome blocks) first GPU run: its tests, the GPU suite, then C5 A/B on one box
# (default threaded vs m16_cs_thread=0) and a rocprofv3 kernel summary of the threaded C5 bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "cs16_threaded or c5_bench_decode or per_stripe_route or reenc or route" > gpurun_out/t_first.log 2>&1 || { tail -30 gpurun_out/t_first.log; exit 1; }
tail -1 gpurun_out/t_first.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_suite.log 2>&1 || { tail -30 gpurun_out/t_suite.log; exit 1; }
tail -1 gpurun_out/t_suite.log
for thr in 1 0 1; do
timeout -k 10 300 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 20 --no-cpu --opt m16_cs_thread=$thr > gpurun_out/t_c5_$thr.log 2>&1 || { tail -5 gpurun_out/t_c5_$thr.log; exit 1; }
echo "thr=$thr"; tail -1 gpurun_out/t_c5_$thr.log | cut -c1-200
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t_prof_c5 -o run -- python3 bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 10 --no-cpu > gpurun_out/t_prof_c5.log 2>&1 || exit 1
find gpurun_out/t_prof_c5 -name "*kernel_stats.csv" -exec head -8 {} \;
timeout -k 10 300 python -u scripts/bench_patterns_c5.py 1024 > gpurun_out/t_patterns_c5.log 2>&1 || { tail -5 gpurun_out/t_patterns_c5.log; exit 1; }
cat gpurun_out/t_patterns_c5.log
