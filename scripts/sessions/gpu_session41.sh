set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt41.log 2>&1 || { tail -30 gpurun_out/pt41.log; exit 1; }
tail -1 gpurun_out/pt41.log
timeout -k 10 300 ./scripts/bench_dropin 4096 1024 1024 16 && timeout -k 10 300 ./scripts/bench_dropin 300 64 65536 16
