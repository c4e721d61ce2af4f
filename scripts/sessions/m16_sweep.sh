set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rt in 64 32 16; do
  RS_AMD_M16_RT=$rt timeout -k 10 300 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 512 --no-cpu --steps 2 --warmup 1 > gpurun_out/m16_$rt.log 2>&1
  echo "rt=$rt rc=$? $(tail -1 gpurun_out/m16_$rt.log | cut -c1-200)"
done
