#!/bin/bash
# Round 3: computed-jump blocks vs gpr-indexed lookups (scripts/ubench/gen_jump.py).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/ubench/bin/jump_bench > gpurun_out/r3_jump_bench.log 2>&1 || { cat gpurun_out/r3_jump_bench.log; exit 1; }
cat gpurun_out/r3_jump_bench.log
