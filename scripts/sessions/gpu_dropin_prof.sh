#!/bin/bash
# Kernel + copy timeline of scripts/bench_dropin at the C3 shape (rocprofv3 SQLite output).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_dropin -o run \
    -- ./scripts/bench_dropin ${1:-128 32 65536 32} > gpurun_out/prof_dropin.log 2>&1
