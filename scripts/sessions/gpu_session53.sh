set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "xor_kernel or config3 or config2 or golden_batch" > gpurun_out/pt53.log 2>&1 || { tail -25 gpurun_out/pt53.log; exit 1; }
tail -1 gpurun_out/pt53.log
timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/bench53.log 2>&1 || { tail -5 gpurun_out/bench53.log; exit 1; }
tail -2 gpurun_out/bench53.log
