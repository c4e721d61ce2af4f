set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_pmc_xj.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --profile-only > gpurun_out/prof16.log 2>&1
echo "prof rc=$?"
