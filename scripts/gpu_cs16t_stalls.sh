#!/bin/bash
# Where k_cs16t's wave cycles go at C5 (SQ busy / wait / issue-stall, instruction fetch and cache,
# clock): one rocprofv3 --pmc pass per counter group over `bench.py --profile-only` (C5, 1024 stripes).
# Summarise with scripts/cs16t_stalls.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/cs16t_stalls
mkdir -p $D
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $D/p$i -o run -- python3 bench.py --profile-only --steps 2 --warmup 2 --k 4096 --r 1024 --symbol 1024 --stripes 1024 > $D/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
