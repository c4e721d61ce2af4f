#!/bin/bash
# Round-2 GPU check: the -m gpu suite, then the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r2_bench.log 2>&1
