#!/bin/bash
# C5 decode at t = 32 and t = 1024: dense GF(2^16) kernels vs the syndrome route (m16_route=2 forces
# the route for every shape; m16_route_min_bytes=0 takes it from the first launch).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="python -u bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 5 --warmup 2 --no-cpu"
for t in ${TS:-32 1024}; do
  timeout -k 10 300 $B --t $t --opt m16_route=0 > gpurun_out/c5_t${t}_dense.log 2>&1 || exit 1
  timeout -k 10 300 $B --t $t --opt m16_route=2 --opt m16_route_min_bytes=0 > gpurun_out/c5_t${t}_route.log 2>&1 || exit 1
  for m in dense route; do
    echo "t=$t $m $(python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/c5_t${t}_$m.log') if x.startswith('{')][-1]; print(l['value'], l['encode_ms'], l['decode_ms'], l['config']['kernel'], l['parity'])")" | tee -a gpurun_out/c5_t.log
  done
done
