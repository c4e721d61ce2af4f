set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "decode_batch" > gpurun_out/pt30.log 2>&1; rc=$?
tail -3 gpurun_out/pt30.log
exit $rc
