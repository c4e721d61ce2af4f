set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt40.log 2>&1 || { tail -30 gpurun_out/pt40.log; exit 1; }
tail -1 gpurun_out/pt40.log
timeout -k 10 300 python scripts/bench_c5_calls.py > gpurun_out/c5calls.log 2>&1 || { tail -5 gpurun_out/c5calls.log; exit 1; }
grep '^{' gpurun_out/c5calls.log
