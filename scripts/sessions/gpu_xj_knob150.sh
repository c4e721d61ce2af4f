#!/bin/bash
# C3 bench A/B of one XOR-kernel knob at the default 150 timed steps: KNOB=VALUE vs KNOB=BASE, alternating, twice.
# usage: gpu_xj_knob150.sh RS_XJ_NAME VALUE BASE
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do for v in "$3" "$2"; do
  env $1=$v timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/k150_${v}_${i}.log 2>&1 || exit 1
  echo "$1=$v run=$i $(python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/k150_${v}_${i}.log') if x.startswith('{')][-1]; print(l['value'], l['encode_ms'], l['decode_ms'], l['parity'])")" | tee -a gpurun_out/k150.log
done; done
