#!/bin/bash
# After an XOR-kernel default change: A/B against the previous default, PMC traffic of both legs of
# the new kernels, the full GPU suite.  usage: gpu_r2_xjclose.sh KNOB=OLDVALUE
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/sessions/gpu_xj_multi.sh "$1" || exit 1
TR=tr bash scripts/gpu_traffic.sh || exit 1
grep -E '"bench_kernel"|traffic_bytes' gpurun_out/traffic.json
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/xc_suite.log 2>&1 || { tail -30 gpurun_out/xc_suite.log; exit 1; }
tail -1 gpurun_out/xc_suite.log
