set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof68 -o run -- python3 scripts/bench_patterns_c5.py 64 > gpurun_out/prof68.log 2>&1 || { tail -20 gpurun_out/prof68.log; exit 1; }
grep distinct gpurun_out/prof68.log
cut -c1-150 gpurun_out/prof68/run_kernel_stats.csv | head -8
