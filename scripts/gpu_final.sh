#!/bin/bash
# Round-end measurement set: GPU tests, smoke, PMC traffic of both bench legs, the bench line (with
# traffic + CPU baseline), and the rocprofv3 kernel stats of the same bench. Copy the results you keep
# from gpurun_out/ into profiles/ afterwards (gpurun_out/traffic.json -> profiles/traffic.json).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt_final.log 2>&1 || { tail -30 gpurun_out/pt_final.log; exit 1; }
tail -1 gpurun_out/pt_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -5 gpurun_out/smoke_final.log; exit 1; }
bash scripts/gpu_traffic.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/final_bench.log 2>&1 || { tail -5 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/final_prof.log 2>&1 || exit 1
tail -1 gpurun_out/final_prof.log
