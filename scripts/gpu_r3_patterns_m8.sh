#!/bin/bash
# GF(256) per-stripe patterns (C3 shape, scripts/bench_patterns.py) on the final tree, after the batch
# decode tests.
set -u
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/patterns_m8
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "decode_batch or golden_batch or edge_empty" > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 t32info > $D/t32info.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 rand > $D/rand.log 2>&1 || exit 1
cat $D/t32info.log $D/rand.log | grep '^{'
