set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc8
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc8/avail.txt 2>&1; echo "list rc=$?"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_MISC SQ_IFETCH_LEVEL SQ_INST_CYCLES_SALU"; do
  for mode in 2 11; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d gpurun_out/pmc8/p${i}_m$mode -o run -- python3 scripts/pmc_one.py $mode 1024 > gpurun_out/pmc8/p${i}_m$mode.log 2>&1
    rc=$?; echo "pass $i mode $mode rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
exit 0
