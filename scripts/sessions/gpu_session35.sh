# C2 (1024 stripes) and C5 (1024 stripes) with CPU baselines.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --k 10 --r 4 --symbol 4096 --stripes 1024 --steps 20 --warmup 3 > gpurun_out/c2_1024.log 2>&1 || exit 1
grep '^{' gpurun_out/c2_1024.log | cut -c1-200
timeout -k 10 600 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 2 --warmup 1 --cpu-stripes 32 --cpu-seconds 10 > gpurun_out/c5_1024.log 2>&1 || exit 1
grep '^{' gpurun_out/c5_1024.log | cut -c1-200
exit 0
