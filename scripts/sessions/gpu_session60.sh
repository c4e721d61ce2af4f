set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
{ timeout -k 10 120 ./scripts/bench_dropin 4096 1024 1024 16 && timeout -k 10 120 ./scripts/bench_dropin && timeout -k 10 120 ./scripts/bench_dropin 10 4 4096 64; } > gpurun_out/dropin60.log 2>&1; rc=$?
cat gpurun_out/dropin60.log
exit $rc
