#!/bin/bash
# rsg_symbol_ops on the GPU: its tests, then scripts/bench_symbol_ops.py over batch shapes (default policy, and
# with RS_AMD_SYMOP_WAVES=1, i.e. no chain splitting, for the A/B). Output gpurun_out/${OUT:-symops}/.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
D=gpurun_out/${OUT:-symops}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "symbol_ops" --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?; tail -2 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/bench_symbol_ops.py > $D/bench.log 2>&1 || exit 1
RS_AMD_SYMOP_WAVES=1 timeout -k 10 120 python -u scripts/bench_symbol_ops.py > $D/bench_w1.log 2>&1 || exit 1
grep '^{' $D/bench.log $D/bench_w1.log | cut -c1-200
