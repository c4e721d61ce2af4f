set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "syndrome_route or per_stripe or distinct_patterns or back_to_back" > gpurun_out/pt54.log 2>&1 || { tail -40 gpurun_out/pt54.log; exit 1; }
tail -3 gpurun_out/pt54.log
timeout -k 10 400 python scripts/bench_patterns.py 4096 t32info > gpurun_out/bp54a.log 2>&1 || { tail -5 gpurun_out/bp54a.log; exit 1; }
cat gpurun_out/bp54a.log
timeout -k 10 400 python scripts/bench_patterns.py 4096 random > gpurun_out/bp54b.log 2>&1 || { tail -5 gpurun_out/bp54b.log; exit 1; }
cat gpurun_out/bp54b.log
