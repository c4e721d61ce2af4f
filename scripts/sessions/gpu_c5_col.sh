#!/bin/bash
# GF(2^16) route block layout A/B (option m16_cs_col: 256 = 4 tiles per 256-byte column block, the
# default; 1024 = the round-1/2 layout, one tile per 1 KiB block): C5 parity tests, the C5 bench line
# with each layout twice, then PMC traffic of both legs with the default.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5col
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "m16 or c5 or route or reenc or golden" --timeout 300 --timeout-method thread > gpurun_out/c5col/suite.log 2>&1 || { tail -30 gpurun_out/c5col/suite.log; exit 1; }
tail -1 gpurun_out/c5col/suite.log
for i in 1 2; do for v in 256 1024; do
  timeout -k 10 300 python -u bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 20 --no-cpu --opt m16_cs_col=$v > gpurun_out/c5col/b_${v}_${i}.log 2>&1 || exit 1
  echo "col=$v run=$i $(python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/c5col/b_${v}_${i}.log') if x.startswith('{')][-1]; print(l['value'], l['encode_ms'], l['decode_ms'], l['parity'])")" | tee -a gpurun_out/c5col/sweep.log
done; done
TR=c5tr bash scripts/gpu_traffic.sh --k 4096 --r 1024 --symbol 1024 --stripes 1024 ${C5_TRAFFIC_OPT:-} || exit 1
cat gpurun_out/c5traffic.json | grep -E '"leg"|traffic_bytes'
