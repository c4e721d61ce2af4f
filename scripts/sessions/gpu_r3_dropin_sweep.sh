#!/bin/bash
# Round 3: registered-symbol drop-in path, column chunks per call (RS_AMD_REG_CHUNKS) at C3.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for ch in 1 2; do
  echo "chunks=$ch" >> gpurun_out/r3_dropin_sweep.log
  RS_AMD_REG_CHUNKS=$ch RS_AMD_PINNED_SEQ=0 timeout -k 10 120 ./scripts/bench_dropin 128 32 65536 64 >> gpurun_out/r3_dropin_sweep.log || exit 1
done
cat gpurun_out/r3_dropin_sweep.log
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "drop_in" > gpurun_out/r3_dropin_tests2.log 2>&1 || { tail -30 gpurun_out/r3_dropin_tests2.log; exit 1; }
tail -1 gpurun_out/r3_dropin_tests2.log
