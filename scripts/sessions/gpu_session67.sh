set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt67.log 2>&1 || { tail -40 gpurun_out/pt67.log; exit 1; }
tail -1 gpurun_out/pt67.log
{ timeout -k 10 120 ./scripts/bench_dropin 128 32 65536 32 && timeout -k 10 120 ./scripts/bench_dropin 4 2 256 256 && timeout -k 10 120 ./scripts/bench_dropin 10 4 4096 64 && timeout -k 10 120 ./scripts/bench_dropin 4096 1024 1024 32 && timeout -k 10 120 ./scripts/bench_dropin 128 32 65536 32; } > gpurun_out/dropin67.log 2>&1; rc=$?
cat gpurun_out/dropin67.log
cat /proc/loadavg
exit $rc
