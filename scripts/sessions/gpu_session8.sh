set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench/issue_bench > gpurun_out/issue_bench.log 2>&1; rc=$?; echo "issue rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_traffic.sh; echo "traffic rc=$?"
