#!/bin/bash
# GPU suite on the current tree (one process, per-test time limit), then the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${CHK:-r4c}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $D/pytest_gpu.log 2>&1
rc=$?; tail -3 $D/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > $D/bench_c3.log 2>&1 || { tail -5 $D/bench_c3.log; exit 1; }
grep '^{' $D/bench_c3.log | cut -c1-400
