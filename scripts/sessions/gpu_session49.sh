set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_reference_programs.py -x -q -m gpu --timeout 300 --timeout-method thread -k "drop_in or reference" > gpurun_out/pt49.log 2>&1 || { tail -20 gpurun_out/pt49.log; exit 1; }
tail -1 gpurun_out/pt49.log
timeout -k 10 120 ./scripts/bench_dropin && timeout -k 10 120 ./scripts/bench_dropin 4096 1024 1024 16 && timeout -k 10 120 ./scripts/bench_dropin 10 4 4096 64 && timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 1024 | grep -o "\"value\": [0-9.]*"
