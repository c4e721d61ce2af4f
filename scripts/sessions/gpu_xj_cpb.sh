#!/bin/bash
# Column-loop A/B (RS_XJ_CPB, rs_xj.cpp): the C3 bench line at cpb = default / 2 / 4 / 8 / 16, twice,
# then the GPU suite with the loop on (every XOR-kernel parity test through the looped kernels).
# usage: gpu_xj_cpb.sh [suite-cpb]
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cpb
for i in 1 2; do for v in default 2 4 16; do
  if [ "$v" = default ]; then E="-u RS_XJ_CPB"; else E="RS_XJ_CPB=$v"; fi
  env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu > gpurun_out/cpb/c3_${v}_${i}.log 2>&1 || exit 1
  echo "CPB=$v run=$i $(python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/cpb/c3_${v}_${i}.log') if x.startswith('{')][-1]; print(l['value'], l['encode_ms'], l['decode_ms'], l['parity'], l['roofline']['frac'])")" | tee -a gpurun_out/cpb/sweep.log
done; done
RS_XJ_CPB=${1:-4} timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cpb/suite.log 2>&1
rc=$?; tail -3 gpurun_out/cpb/suite.log; exit $rc
