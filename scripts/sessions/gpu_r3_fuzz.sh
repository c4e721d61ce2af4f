#!/bin/bash
# Round 3: parity fuzz over the new paths, then every family.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/fuzz_parity.py 3031 300 ps16,orbit,dropin_reg > gpurun_out/r3_fuzz_new.jsonl 2>&1 || { tail -5 gpurun_out/r3_fuzz_new.jsonl; exit 1; }
tail -1 gpurun_out/r3_fuzz_new.jsonl
timeout -k 10 400 python -u scripts/fuzz_parity.py 3032 300 > gpurun_out/r3_fuzz_all.jsonl 2>&1 || { tail -5 gpurun_out/r3_fuzz_all.jsonl; exit 1; }
tail -1 gpurun_out/r3_fuzz_all.jsonl
