#!/bin/bash
# Closing check on the current tree: the GPU suite (one process), smoke, the default bench line and a parity fuzz
# over every family (FUZZ_S seconds, default 540). Output gpurun_out/${CLOSE:-close}/.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
D=gpurun_out/${CLOSE:-close}; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?; tail -2 $D/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python3 -u bench.py > $D/bench_c3.log 2>&1 || { tail -5 $D/bench_c3.log; exit 1; }
grep '^{' $D/bench_c3.log | cut -c1-200
timeout -k 10 $(( ${FUZZ_S:-540} + 120 )) python3 -u scripts/fuzz_parity.py ${FUZZ_SEED:-9099} ${FUZZ_S:-540} > $D/fuzz.log 2>&1 || { tail -20 $D/fuzz.log; exit 1; }
tail -1 $D/fuzz.log
