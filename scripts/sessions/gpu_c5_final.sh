#!/bin/bash
# C5 (k=4096, r=1024, 1 KiB, 1024 stripes): bench line (syndrome route, compute roofline), rocprofv3
# kernel statistics, and one PMC pass of instruction counts to check rsg_last_work.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/c5final
mkdir -p $D
ARGS="--k 4096 --r 1024 --symbol 1024 --stripes 1024"
timeout -k 10 300 python3 -u bench.py $ARGS --steps 5 --warmup 2 --no-cpu > $D/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/stats -o run -- python3 bench.py $ARGS --steps 3 --warmup 1 --no-cpu --profile-only > $D/stats.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $D/pmc -o run -- python3 bench.py --k 4096 --r 1024 --symbol 1024 --stripes 256 --steps 1 --warmup 0 --no-cpu --profile-only > $D/pmc.log 2>&1
find $D -name "*.csv" | head -20
