set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/bench_dropin 4096 1024 1024 16 > gpurun_out/dropin_c5.log 2>&1 || { cat gpurun_out/dropin_c5.log; exit 1; }
timeout -k 10 300 ./scripts/bench_dropin > gpurun_out/dropin_c3.log 2>&1 || exit 1
cat gpurun_out/dropin_c5.log gpurun_out/dropin_c3.log
