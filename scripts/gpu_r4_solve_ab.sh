#!/bin/bash
# A/Bs of the V = 1 GF(256) solve kernels (per-stripe route 2 over 4096 C3 stripes, scripts/bench_patterns.py;
# one shared pattern on the generic kernel). usage: gpu_r4_solve_ab.sh MODE
#   check  GF(256) GPU tests, phase stamps (diagnostic library, scripts/gpu_stamps_v1.py), per-stripe t32info /
#          rand and the generic kernel at m8_mode 18 / 20, two reps (the round-4 output-stage and prologue
#          changes were measured with it)
#   v1h    solve kernel 0 (two tables) vs 3 / 4 / 5 (one table; inputs converted 1 / 2 / 4 per LDS round trip),
#          then SQ PMC passes for kernels 0 and 4
#   noidx  index-switch ceiling (diagnostic library; wrong results): solve kernel 0 vs 6, generic m8_mode
#          18 vs 19 vs 20
#   cpb    column chunks per workgroup of solve kernel 0 (option m8_ps_cpb) 1 / 2 / 4 / 8 / 16
#   sqc    scalar-cache counters (SQC_DCACHE_*) of the per-stripe solve vs one shared pattern
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
MODE=${1:?mode}
D=gpurun_out/${PS8:-solve_$MODE}
mkdir -p $D
DIAG=$PWD/reed-solomon_amd/librs_amd_diag.so
run() {  # run LABEL ARGS... with the environment already exported by the caller
  local label=$1; shift
  timeout -k 10 300 python3 -u scripts/bench_patterns.py "$@" > $D/$label.log 2>&1 || { tail -5 $D/$label.log; exit 1; }
  echo "$label $(grep -o '"ms": [0-9.]*' $D/$label.log) $(grep -o '"restored": [a-z]*' $D/$label.log)"
}
tests() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "$1" > $D/tests.log 2>&1
  local rc=$?; tail -1 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
}
pmc() {  # pmc DIR "COUNTERS" ARGS...
  local dir=$1 grp=$2; shift 2
  timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $D/$dir -o run -- python3 scripts/bench_patterns.py "$@" > $D/$dir.log 2>&1
  local rc=$?; [ $rc -ne 0 ] && { tail -3 $D/$dir.log; exit $rc; }
}
case $MODE in
check)
  tests "golden_batch or decode_batch or edge_empty or reenc or drop_in"
  RS_AMD_LIB=$DIAG timeout -k 10 300 python3 -u scripts/gpu_stamps_v1.py > $D/stamps.log 2>&1 || exit 1
  grep '^{' $D/stamps.log
  for rep in 1 2; do
    for pat in t32info rand; do run ps_${pat}_$rep 4096 $pat device_plans_syndrome; done
    for mm in 18 20; do RS_PS8_M8MODE=$mm run g${mm}_$rep 4096 t32info one_pattern_generic; done
  done ;;
v1h)
  tests "decode_batch_syndrome_route"
  for rep in 1 2; do for kn in 0 3 4 5; do for pat in t32info rand; do
    RS_PS8_KERNEL=$kn run k${kn}_${pat}_$rep 4096 $pat device_plans_syndrome
  done; done; done
  for kn in 0 4; do
    export RS_PS8_KERNEL=$kn
    pmc pmc_k$kn/p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" 4096 t32info device_plans_syndrome
    pmc pmc_k$kn/p2 "SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" 4096 t32info device_plans_syndrome
    echo "== kernel $kn"; python3 scripts/pmc_summary.py $D/pmc_k$kn "k_apply_m8_v1<"
  done ;;
noidx)
  export RS_AMD_LIB=$DIAG
  for rep in 1 2; do
    for kn in 0 6; do RS_PS8_KERNEL=$kn run k${kn}_$rep 4096 t32info device_plans_syndrome; done
    for mm in 18 19 20; do RS_PS8_M8MODE=$mm run g${mm}_$rep 4096 t32info one_pattern_generic; done
  done ;;
cpb)
  tests "decode_batch_syndrome_route or golden_batch"
  for rep in 1 2; do for cpb in 1 2 4 8 16; do for pat in t32info rand; do
    RS_PS8_CPB=$cpb run c${cpb}_${pat}_$rep 4096 $pat device_plans_syndrome
  done; done; done ;;
sqc)
  C="SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE"
  pmc ps "$C" 4096 t32info device_plans_syndrome
  RS_PS8_M8MODE=18 pmc one "$C" 4096 t32info one_pattern_generic
  echo "== per-stripe"; python3 scripts/pmc_summary.py $D/ps "k_apply_m8_v1<"
  echo "== one pattern"; python3 scripts/pmc_summary.py $D/one "k_apply_m8_v1<" ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
