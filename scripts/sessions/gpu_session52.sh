set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "host_memory or drop_in" > gpurun_out/pt52.log 2>&1 || { tail -25 gpurun_out/pt52.log; exit 1; }
tail -1 gpurun_out/pt52.log
timeout -k 10 600 python scripts/bench_host.py > gpurun_out/bench_host.log 2>&1 || { tail -5 gpurun_out/bench_host.log; exit 1; }
tail -1 gpurun_out/bench_host.log
