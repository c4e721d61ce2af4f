#!/bin/bash
# Where the C3 encode XOR kernel's wave cycles go (SQ busy / wait / issue-stall / per-unit active
# cycles, instruction fetch): one rocprofv3 --pmc pass per counter group over scripts/pmc_xj.py
# (1024 stripes, 3 encode launches). Summarise with scripts/xj_stalls.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/xj_stalls
mkdir -p $D
timeout -s KILL 60 rocprofv3 --list-avail > $D/avail.txt 2>&1; echo "list rc=$?"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $D/p$i -o run -- python3 scripts/pmc_xj.py jit 1024 enc > $D/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
