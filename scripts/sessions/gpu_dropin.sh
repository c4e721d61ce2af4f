#!/bin/bash
# Per-call drop-in path on the GPU box: the drop-in parity tests, then scripts/bench_dropin at the C3
# and C5 shapes with page-locked arenas (default) and with pageable symbols (RS_AMD_PINNED_SEQ=0).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/reed-solomon_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "drop_in or dropin" > gpurun_out/dropin_tests.log 2>&1 || { tail -30 gpurun_out/dropin_tests.log; exit 1; }
tail -2 gpurun_out/dropin_tests.log
for shape in "128 32 65536 32" "4096 1024 4096 8" "4 2 256 512" "10 4 4096 512"; do
    timeout -k 10 120 ./scripts/bench_dropin $shape | tee -a gpurun_out/dropin_bench.log || exit 1
    RS_AMD_PINNED_SEQ=0 timeout -k 10 120 ./scripts/bench_dropin $shape | tee -a gpurun_out/dropin_bench.log || exit 1
done
if [ -n "$DROPIN_PROF" ]; then
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
    timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_dropin -o run \
        -- ./scripts/bench_dropin 128 32 65536 32 > gpurun_out/prof_dropin.log 2>&1 || exit 1
fi
