#!/bin/bash
# Round-4 close, part A: the whole GPU suite (one process), smoke, the default bench line (C3 with the
# port CPU baseline) and the rocprofv3 kernel summary of the same bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${CLOSE:-r4close}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?; tail -2 $D/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python3 -u bench.py > $D/bench_c3.log 2>&1 || { tail -5 $D/bench_c3.log; exit 1; }
grep '^{' $D/bench_c3.log | cut -c1-400
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c3 -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $D/prof_c3.log 2>&1 || exit 1
grep '^{' $D/prof_c3.log | cut -c1-200
