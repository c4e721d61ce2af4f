#!/bin/bash
# Per-phase VALU / SALU of the C3 XOR kernels (rows / subset tables / finish) from SQ counters: the
# diagnostic library's timing ablations (RS_XJ_ABLATE 1 = no finish, 2 = no rows, 4 = no tables)
# against the full kernel, for the encode and the bench-pattern decode kernel (scripts/pmc_xj.py,
# 1024 stripes, 3 launches each). One rocprofv3 --pmc pass per (op, ablation).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/xj_phases
mkdir -p $D
export RS_AMD_LIB=$PWD/reed-solomon_amd/librs_amd_diag.so
for op in enc dec; do
  for ab in 0 1 2 4; do
    RS_XJ_ABLATE=$ab timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv \
        --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        -d $D/${op}_a$ab -o run -- python3 scripts/pmc_xj.py jit 1024 $op > $D/${op}_a$ab.log 2>&1
    rc=$?; echo "$op ablate $ab rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
