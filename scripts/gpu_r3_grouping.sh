#!/bin/bash
# Host-side pattern grouping rewrite (hash + vectorised counts): the batch-decode GPU tests, then the
# per-stripe C5 route's wall time and kernel breakdown (scripts/prof_ps16.py under rocprofv3).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${1:-grouping}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "decode_batch or golden_batch or edge_empty or drop_in" > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 -u scripts/prof_ps16.py 1024 > $D/prof.log 2>&1
rc=$?; grep -E "^run|restored" $D/prof.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_patterns_c5.py 1024 > $D/patterns.log 2>&1
rc=$?; cat $D/patterns.log; exit $rc
