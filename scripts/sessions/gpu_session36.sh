set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "shapes or m16" > gpurun_out/pt36.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/pt36.log | head -30; tail -1 gpurun_out/pt36.log
exit $rc
