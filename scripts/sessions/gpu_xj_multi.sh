#!/bin/bash
# C3 bench (20 timed steps) over several XOR-kernel knob settings on one box, each setting twice,
# interleaved with the default. usage: gpu_xj_multi.sh "K1=V1 K2=V2" "K3=V3" ...  ("default" = no knob)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/multi
for i in 1 2; do for cfg in default "$@"; do
  tag=$(echo "$cfg" | tr ' =' '_-')
  if [ "$cfg" = default ]; then E=""; else E="$cfg"; fi
  env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu > gpurun_out/multi/${tag}_${i}.log 2>&1 || exit 1
  echo "$cfg run=$i $(python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/multi/${tag}_${i}.log') if x.startswith('{')][-1]; print(l['value'], l['encode_ms'], l['decode_ms'], l['parity'])")" | tee -a gpurun_out/multi/sweep.log
done; done
