set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt61.log 2>&1 || { tail -40 gpurun_out/pt61.log; exit 1; }
tail -1 gpurun_out/pt61.log
{ timeout -k 10 120 ./scripts/bench_dropin 4096 1024 1024 16 && timeout -k 10 120 ./scripts/bench_dropin && timeout -k 10 120 ./scripts/bench_dropin 10 4 4096 64; } > gpurun_out/dropin61.log 2>&1; rc=$?
cat gpurun_out/dropin61.log
exit $rc
