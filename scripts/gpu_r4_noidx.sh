#!/bin/bash
# Index-switch ceiling of the V = 1 GF(256) kernels (diagnostic library; the ablations give wrong
# results): per-stripe solve kernel 0 vs 6 (fixed table registers, no s_set_gpr_idx), one shared pattern
# on the generic kernel m8_mode 18 vs 19 (the same ablation) vs 20, two alternating reps.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export RS_AMD_LIB=$PWD/reed-solomon_amd/librs_amd_diag.so
D=gpurun_out/${PS8:-noidx}
mkdir -p $D
for rep in 1 2; do
  for kn in 0 6; do
    RS_PS8_KERNEL=$kn timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/k${kn}_$rep.log 2>&1 || exit 1
    echo "ps kernel $kn $(grep -o '"ms": [0-9.]*' $D/k${kn}_$rep.log)"
  done
  for mm in 18 19 20; do
    RS_PS8_M8MODE=$mm timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 t32info one_pattern_generic > $D/g${mm}_$rep.log 2>&1 || exit 1
    echo "generic m8_mode $mm $(grep -o '"ms": [0-9.]*' $D/g${mm}_$rep.log)"
  done
done
