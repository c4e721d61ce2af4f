set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof37 -o run -- python3 scripts/bench_c5_calls.py > gpurun_out/c5calls.log 2>&1; rc=$?
grep '^{' gpurun_out/c5calls.log; tail -2 gpurun_out/c5calls.log | cut -c1-300
cut -d, -f1-4 gpurun_out/prof37/run_kernel_stats.csv | head -8
exit $rc
