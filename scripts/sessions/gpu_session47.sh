set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
C5="--k 4096 --r 1024 --symbol 1024 --stripes 512"
for pad in 0 40000 70000; do
  RS_M16_LDS_PAD=$pad timeout -k 10 300 python bench.py --no-cpu --profile-only --steps 2 --warmup 1 $C5 > gpurun_out/pad$pad.log 2>&1 || exit 1
  echo "pad=$pad $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/pad$pad.log)"
  RS_M16_LDS_PAD=$pad timeout -k 10 300 python bench.py --no-cpu --profile-only --steps 2 --warmup 1 $C5 --kernel m16p > gpurun_out/padp$pad.log 2>&1 || exit 1
  echo "plain pad=$pad $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/padp$pad.log)"
done
