set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for kern in m16p auto; do
  timeout -k 10 300 python bench.py --no-cpu --profile-only --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 512 --kernel $kern > gpurun_out/c5_$kern.log 2>&1 || exit 1
  echo "$kern $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/c5_$kern.log)"
done
exit 0
