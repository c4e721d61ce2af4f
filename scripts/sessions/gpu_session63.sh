set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt63.log 2>&1 || { tail -40 gpurun_out/pt63.log; exit 1; }
tail -1 gpurun_out/pt63.log
{ timeout -k 10 120 ./scripts/bench_dropin 4096 1024 1024 32 && timeout -k 10 120 ./scripts/bench_dropin 128 32 65536 32 && timeout -k 10 120 ./scripts/bench_dropin 10 4 4096 64 && timeout -k 10 120 ./scripts/bench_dropin 4 2 256 256; } > gpurun_out/dropin63.log 2>&1; rc=$?
cat gpurun_out/dropin63.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_patterns_c5.py 256 > gpurun_out/bp63.log 2>&1 || { tail -20 gpurun_out/bp63.log; exit 1; }
cat gpurun_out/bp63.log
cat /proc/loadavg
