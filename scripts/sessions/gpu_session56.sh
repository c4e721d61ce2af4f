set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_patterns_c5.py 64 > gpurun_out/bp56.log 2>&1 || { tail -20 gpurun_out/bp56.log; exit 1; }
cat gpurun_out/bp56.log
timeout -k 10 300 python scripts/bench_patterns_c5.py 256 > gpurun_out/bp56b.log 2>&1 || { tail -20 gpurun_out/bp56b.log; exit 1; }
cat gpurun_out/bp56b.log
