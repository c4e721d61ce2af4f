set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u scripts/fuzz_parity.py 2025 300 > gpurun_out/fuzz65.log 2>&1; rc=$?
tail -1 gpurun_out/fuzz65.log
grep -c '"ok": false' gpurun_out/fuzz65.log || true
exit $rc
