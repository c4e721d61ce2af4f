#!/bin/bash
# C3 bench A/B of one XOR-kernel generation knob: KNOB=VALUE vs default (knob unset), alternating,
# twice each.
# usage: gpu_xj_knob.sh RS_XJ_NAME VALUE
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do for v in default "$2"; do
  if [ "$v" = default ]; then E="-u $1"; else E="$1=$v"; fi
  env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu > gpurun_out/knob_${v}_${i}.log 2>&1 || exit 1
  echo "$1=$v run=$i $(python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/knob_${v}_${i}.log') if x.startswith('{')][-1]; print(l['value'], l['encode_ms'], l['decode_ms'], l['parity'])")" | tee -a gpurun_out/knob.log
done; done
