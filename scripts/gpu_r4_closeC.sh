#!/bin/bash
# Round-4 close, part C: the C5 bench line with the merged traffic records, and the registered-symbol
# drop-in fuzz family with the registration checked after the first call (registration on first use).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${CLOSE:-r4close}
mkdir -p $D
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --k 4096 --r 1024 --symbol 1024 --stripes 1024 > $D/bench_c5b.log 2>&1 || { tail -5 $D/bench_c5b.log; exit 1; }
grep '^{' $D/bench_c5b.log | cut -c1-200
timeout -k 10 300 python3 -u scripts/fuzz_parity.py 405 150 dropin_reg,dropin,batch > $D/fuzz_reg.log 2>&1 || { tail -20 $D/fuzz_reg.log; exit 1; }
tail -1 $D/fuzz_reg.log
