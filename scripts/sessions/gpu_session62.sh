set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
{ timeout -k 10 120 ./scripts/bench_dropin 4096 1024 1024 32 && timeout -k 10 120 ./scripts/bench_dropin 4096 1024 1024 32 && timeout -k 10 120 ./scripts/bench_dropin 128 32 65536 32; } > gpurun_out/dropin62.log 2>&1; rc=$?
cat gpurun_out/dropin62.log
nproc; cat /proc/loadavg
exit $rc
