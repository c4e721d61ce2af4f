#!/bin/bash
# Round-end measurement set on the current tree: the whole GPU suite (one process), smoke, the default bench
# line (C3, with the port CPU baseline and its calibration, and the extra legs: per-stripe patterns, host
# memory, C2 / C5, batched symbol ops) and its rocprofv3 kernel summary, PMC traffic of both bench legs at
# C3, C5 and C2 (separate FETCH_SIZE / WRITE_SIZE passes, scripts/gpu_traffic.sh), the C5 bench line, and
# with FUZZ=1 one mixed parity fuzz run. Afterwards merge gpurun_out/$CLOSE/c*affic.json into
# profiles/traffic.json (records are keyed by kernel source hash; rerun the bench once they are in) and copy
# the logs you keep into profiles/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${CLOSE:-final}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?; tail -2 $D/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python3 -u bench.py > $D/bench_c3.log 2>&1 || { tail -5 $D/bench_c3.log; exit 1; }
grep '^{' $D/bench_c3.log | cut -c1-300
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c3 -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $D/prof_c3.log 2>&1 || exit 1
TR=${CLOSE:-final}/c3 bash scripts/gpu_traffic.sh || exit 1
TR=${CLOSE:-final}/c5 bash scripts/gpu_traffic.sh --k 4096 --r 1024 --symbol 1024 --stripes 1024 || exit 1
TR=${CLOSE:-final}/c2 bash scripts/gpu_traffic.sh --k 10 --r 4 --symbol 4096 --stripes 1024 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --k 4096 --r 1024 --symbol 1024 --stripes 1024 --no-extras > $D/bench_c5.log 2>&1 || { tail -5 $D/bench_c5.log; exit 1; }
grep '^{' $D/bench_c5.log | cut -c1-300
if [ "${FUZZ:-0}" = 1 ]; then
  timeout -k 10 360 python3 -u scripts/fuzz_parity.py 606 240 > $D/fuzz.log 2>&1 || { tail -20 $D/fuzz.log; exit 1; }
  tail -1 $D/fuzz.log
fi
