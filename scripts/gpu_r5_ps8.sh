#!/bin/bash
# Round-5 A/Bs of the GF(256) per-stripe decode (route 2, 4096 C3 stripes, scripts/bench_patterns.py).
# usage: gpu_r5_ps8.sh MODE
#   rec    solve kernel 0 vs the diagnostic one-record-round-trip ablation 8 (wrong results): how much of the
#          step is the high-half record load's exposed latency
#   kern   the production solve vs diagnostic solve kernels KERNS (default 1), t32info and rand
#   base   the production route alone (t32info and rand), two reps
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
MODE=${1:?mode}
D=gpurun_out/${PS8:-r5_ps8_$MODE}
mkdir -p $D
DIAG=$PWD/reed-solomon_amd/librs_amd_diag.so
run() {  # run LABEL ARGS... with the environment already exported by the caller
  local label=$1; shift
  timeout -k 10 300 python3 -u scripts/bench_patterns.py "$@" > $D/$label.log 2>&1 || { tail -5 $D/$label.log; exit 1; }
  echo "$label $(grep -o '"ms": [0-9.]*' $D/$label.log | head -1) $(grep -o '"restored": [a-z]*' $D/$label.log | head -1)"
}
case $MODE in
rec)
  for rep in 1 2; do
    run rel_$rep 4096 t32info device_plans_syndrome
    for kern in 0 8; do RS_AMD_LIB=$DIAG RS_PS8_KERNEL=$kern run k${kern}_$rep 4096 t32info device_plans_syndrome; done
  done ;;
abl)   # per-stripe solve fixed costs: ablation bits 1 no table copy, 2 no output conversion, 4 no old-value loads
  for rep in 1 2; do for ab in 0 1 2 4 7; do
    RS_AMD_LIB=$DIAG RS_PS8_ABLATE=$ab run a${ab}_$rep 4096 t32info device_plans_syndrome
  done; done ;;
prof)  # rocprofv3 kernel split of the production route (t32info, 4096 stripes)
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
  grep '^{' $D/prof.log; head -8 $D/prof/run_kernel_stats.csv | cut -c1-160 ;;
baseprof)  # the production route twice, then its rocprofv3 kernel split
  for rep in 1 2; do for pat in t32info rand; do run ${pat}_$rep 4096 $pat device_plans_syndrome; done; done
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
  grep '^{' $D/prof.log; head -6 $D/prof/run_kernel_stats.csv | cut -c1-160 ;;
kern)  # the production solve against solve kernels $KERNS (m8_ps_kernel values; library $KLIB, default the
       # diagnostic one), t32info and rand
  for rep in 1 2; do
    run rel_t32_$rep 4096 t32info device_plans_syndrome
    run rel_rand_$rep 4096 rand device_plans_syndrome
    for kern in ${KERNS:-1}; do
      RS_AMD_LIB=${KLIB:-$DIAG} RS_PS8_KERNEL=$kern run k${kern}_t32_$rep 4096 t32info device_plans_syndrome
      RS_AMD_LIB=${KLIB:-$DIAG} RS_PS8_KERNEL=$kern run k${kern}_rand_$rep 4096 rand device_plans_syndrome
    done
  done ;;
kprof)  # rocprofv3 kernel split with solve kernel $KERN (release library)
  RS_PS8_KERNEL=${KERN:-9} timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
  grep '^{' $D/prof.log; head -6 $D/prof/run_kernel_stats.csv | cut -c1-160 ;;
base)
  for rep in 1 2; do for pat in t32info rand; do run ${pat}_$rep 4096 $pat device_plans_syndrome; done; done ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
