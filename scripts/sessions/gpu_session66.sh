set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof66 -o run -- ./scripts/bench_dropin 128 32 65536 32 > gpurun_out/prof66.log 2>&1 || { tail -20 gpurun_out/prof66.log; exit 1; }
tail -1 gpurun_out/prof66.log
cut -c1-160 gpurun_out/prof66/run_kernel_stats.csv
