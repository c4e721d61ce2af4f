# Effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) of the encode kernel, normal vs aliased.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export RS_AMD_LIB=$GRAFT_REPO_ROOT/reed-solomon_amd/librs_amd_diag.so  # RS_XJ_ALIAS: diagnostic build only
D=gpurun_out/clock
mkdir -p $D
for v in 0 1; do
  RS_XJ_ALIAS=$v timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $D/a$v -o run -- python3 scripts/pmc_xj.py jit 4096 > $D/a$v.log 2>&1
  echo "alias $v rc=$?"
done
