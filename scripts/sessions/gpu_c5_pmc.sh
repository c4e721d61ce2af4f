#!/bin/bash
# PMC passes over one C5 encode + decode (syndrome route): issue / stall counters of k_cs16 and the
# second stage. Each pass is its own short run (rocprofv3 does not split counters over passes).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/c5pmc
mkdir -p $D
CMD="python3 bench.py --k 4096 --r 1024 --symbol 1024 --stripes 256 --steps 1 --warmup 0 --no-cpu --profile-only"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $D/p1 -o run -- $CMD > $D/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_IFETCH SQ_WAIT_INST_LDS -d $D/p2 -o run -- $CMD > $D/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d $D/p3 -o run -- $CMD > $D/p3.log 2>&1
find $D -name "*counter_collection.csv" | while read f; do cp "$f" $D/$(basename $(dirname $(dirname "$f")))_$(basename "$f"); done
ls -R $D | head -40
