#!/bin/bash
# C5 route: shape tests over both block layouts, PMC traffic of both legs (default layout), bench line.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "m16_kernel_shapes or reenc or golden" --timeout 300 --timeout-method thread > gpurun_out/c5t_suite.log 2>&1 || { tail -30 gpurun_out/c5t_suite.log; exit 1; }
tail -1 gpurun_out/c5t_suite.log
TR=c5tr bash scripts/gpu_traffic.sh --k 4096 --r 1024 --symbol 1024 --stripes 1024 || exit 1
grep -E '"leg"|traffic_bytes' gpurun_out/c5traffic.json
