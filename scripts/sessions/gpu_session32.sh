set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 bash scripts/gpu_traffic.sh rs_xj rs_xj > gpurun_out/traffic.log 2>&1 || { tail -5 gpurun_out/traffic.log; exit 1; }
cp gpurun_out/traffic.json profiles/traffic.json
timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/bench32.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"traffic": [^,]*' gpurun_out/bench32.log
