set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_reference_programs.py -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pt33.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|exit" gpurun_out/pt33.log | head -20
timeout -k 10 120 ./oracle/_ref/reftests/example > gpurun_out/example.log 2>&1; echo "example rc=$?"; head -c 1500 gpurun_out/example.log
exit $rc
