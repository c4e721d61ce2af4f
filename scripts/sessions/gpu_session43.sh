set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
C5="--k 4096 --r 1024 --symbol 1024 --stripes 1024"
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "m16 or c5_ or wide_r or large_n or max_n" > gpurun_out/pt43.log 2>&1 || { tail -20 gpurun_out/pt43.log; exit 1; }
tail -1 gpurun_out/pt43.log
timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 $C5 > gpurun_out/c5x.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"parity": "[^"]*"' gpurun_out/c5x.log
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d gpurun_out/c5_fetch -o run -- python3 bench.py --no-cpu --profile-only --steps 1 --warmup 1 $C5 > gpurun_out/c5_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d gpurun_out/c5_write -o run -- python3 bench.py --no-cpu --profile-only --steps 1 --warmup 1 $C5 > gpurun_out/c5_write.log 2>&1 || exit 1
