#!/bin/bash
# Round-3 measurement set: GPU suite, smoke, PMC traffic of both legs at C3 and C5, the C3 and C5 bench
# lines, rocprofv3 kernel stats of the default C3 bench and of C5, the C5 per-stripe pattern bench.
# Copy what is kept into profiles/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/f_suite.log 2>&1 || { tail -30 gpurun_out/f_suite.log; exit 1; }
tail -1 gpurun_out/f_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || { tail -5 gpurun_out/f_smoke.log; exit 1; }
tail -1 gpurun_out/f_smoke.log
TR=tr bash scripts/gpu_traffic.sh || exit 1
TR=c5tr bash scripts/gpu_traffic.sh --k 4096 --r 1024 --symbol 1024 --stripes 1024 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/f_bench_c3.log 2>&1 || { tail -5 gpurun_out/f_bench_c3.log; exit 1; }
tail -1 gpurun_out/f_bench_c3.log | cut -c1-300
timeout -k 10 600 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 20 > gpurun_out/f_bench_c5.log 2>&1 || { tail -5 gpurun_out/f_bench_c5.log; exit 1; }
tail -1 gpurun_out/f_bench_c5.log | cut -c1-300
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_prof -o run -- python3 bench.py > gpurun_out/f_prof.log 2>&1 || exit 1
tail -1 gpurun_out/f_prof.log | cut -c1-300
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_prof_c5 -o run -- python3 bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 10 > gpurun_out/f_prof_c5.log 2>&1 || exit 1
tail -1 gpurun_out/f_prof_c5.log | cut -c1-300
timeout -k 10 300 python -u scripts/bench_patterns_c5.py 1024 > gpurun_out/f_patterns_c5.log 2>&1 || { tail -5 gpurun_out/f_patterns_c5.log; exit 1; }
cat gpurun_out/f_patterns_c5.log
