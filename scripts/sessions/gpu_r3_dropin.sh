#!/bin/bash
# Round 3: drop-in per-call path on registered caller symbols (RS_AMD_PINNED_SEQ=0) vs arenas.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "drop_in or symbol_ops or reference_surface" > gpurun_out/r3_dropin_tests.log 2>&1 || { tail -40 gpurun_out/r3_dropin_tests.log; exit 1; }
tail -2 gpurun_out/r3_dropin_tests.log
for shape in "128 32 65536 64" "10 4 4096 256" "4096 1024 4096 16"; do
  RS_AMD_PINNED_SEQ=0 timeout -k 10 120 ./scripts/bench_dropin $shape >> gpurun_out/r3_dropin.jsonl || exit 1
  timeout -k 10 120 ./scripts/bench_dropin $shape >> gpurun_out/r3_dropin.jsonl || exit 1
done
cat gpurun_out/r3_dropin.jsonl
