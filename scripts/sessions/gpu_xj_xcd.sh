#!/bin/bash
# C3 bench with the XOR kernels' XCD-contiguous column remap off / on (RS_XJ_XCD), twice each.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do for x in 0 1; do
  RS_XJ_XCD=$x timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/xcd_${x}_${i}.log 2>&1 || exit 1
  echo "xcd=$x run=$i $(python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/xcd_${x}_${i}.log') if x.startswith('{')][-1]; print(l['value'], l['encode_ms'], l['decode_ms'])")" | tee -a gpurun_out/xcd.log
done; done
