set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ks69.log
for ks in 32 64 16 128; do
  RS_AMD_KSLICES=$ks timeout -k 10 200 python scripts/bench_patterns_c5.py 64 > gpurun_out/ks.log 2>&1 || { tail -5 gpurun_out/ks.log; exit 1; }
  grep stream_plans gpurun_out/ks.log | sed "s/^/ks=$ks /" >> gpurun_out/ks69.log
done
cat gpurun_out/ks69.log
