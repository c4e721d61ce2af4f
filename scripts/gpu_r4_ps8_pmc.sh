#!/bin/bash
# Where the per-stripe GF(256) route's kernels spend their wave cycles (rsg_decode_batch, 4096 C3 stripes,
# all-distinct t = 32 patterns; scripts/bench_patterns.py device_plans_syndrome): SQ busy / wait /
# issue-stall, instruction counts, LDS, clock. One rocprofv3 --pmc pass per counter group; summarise with
# scripts/pmc_summary.py DIR KERNEL.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${PS8:-ps8pmc}
mkdir -p $D
[ -n "${KERN:-}" ] && export RS_PS8_KERNEL=$KERN  # the per-stripe solve kernel (m8_ps_kernel)
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH SQC_ICACHE_MISSES"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $D/p$i -o run -- python3 scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) tail -3 $D/p$i.log; exit $rc;; esac
done
for k in "k_apply_m8_v1<0>" k_apply_m8_pf k_apply_m8_ps_w rs_xj_ k_plan_; do echo "== $k"; python3 scripts/pmc_summary.py $D "$k"; done
