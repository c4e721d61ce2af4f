set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "m16 or golden or per_stripe or distinct_patterns or back_to_back or syndrome" > gpurun_out/pt57.log 2>&1 || { tail -40 gpurun_out/pt57.log; exit 1; }
tail -3 gpurun_out/pt57.log
timeout -k 10 300 python scripts/bench_patterns_c5.py 64 > gpurun_out/bp57a.log 2>&1 || { tail -20 gpurun_out/bp57a.log; exit 1; }
cat gpurun_out/bp57a.log
timeout -k 10 300 python scripts/bench_patterns_c5.py 256 > gpurun_out/bp57b.log 2>&1 || { tail -20 gpurun_out/bp57b.log; exit 1; }
cat gpurun_out/bp57b.log
