set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "m16 or c5_ or wide_r or golden" > gpurun_out/pt38.log 2>&1 || { tail -30 gpurun_out/pt38.log; exit 1; }
tail -1 gpurun_out/pt38.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof38 -o run -- python3 scripts/bench_c5_calls.py > gpurun_out/c5calls.log 2>&1 || exit 1
grep '^{' gpurun_out/c5calls.log
cut -d, -f1-4 gpurun_out/prof38/run_kernel_stats.csv | head -6
timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 1024 > gpurun_out/c5b.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"parity": "[^"]*"' gpurun_out/c5b.log
