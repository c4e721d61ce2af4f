#!/bin/bash
# Round-4 close, part B: PMC traffic of both bench legs at C3 and C5 on the final kernels (separate
# FETCH_SIZE / WRITE_SIZE passes, scripts/gpu_traffic.sh), the C5 bench line, and (FUZZ=1) one mixed parity
# fuzz run (every kernel family, including the registered-symbol drop-in path; run once, not repeated).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${CLOSE:-r4close}
mkdir -p $D
TR=${CLOSE:-r4close}/c3 bash scripts/gpu_traffic.sh || exit 1
TR=${CLOSE:-r4close}/c5 bash scripts/gpu_traffic.sh --k 4096 --r 1024 --symbol 1024 --stripes 1024 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --k 4096 --r 1024 --symbol 1024 --stripes 1024 > $D/bench_c5.log 2>&1 || { tail -5 $D/bench_c5.log; exit 1; }
grep '^{' $D/bench_c5.log | cut -c1-300
if [ "${FUZZ:-0}" = 1 ]; then
  timeout -k 10 420 python3 -u scripts/fuzz_parity.py 404 300 > $D/fuzz.log 2>&1 || { tail -20 $D/fuzz.log; exit 1; }
  tail -2 $D/fuzz.log
fi
