#!/bin/bash
# V = 1 output stage with the tile's 32 output slots loaded once (two SMEM loads) and every xor_dst old
# value loaded before the conversions: GPU tests of the GF(256) paths, then per-stripe solve kernels 0 / 3 /
# 4 (route 2, t32info and rand) and the one-pattern generic kernel (m8_mode 18 / 20), two reps.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${PS8:-store}
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "golden_batch or decode_batch or edge_empty or reenc or drop_in or transform" > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
for rep in 1 2; do
  for kn in 0 3 4; do for pat in t32info rand; do
    RS_PS8_KERNEL=$kn timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 $pat device_plans_syndrome > $D/k${kn}_${pat}_$rep.log 2>&1 || exit 1
    echo "ps kernel $kn $pat $(grep -o '"ms": [0-9.]*' $D/k${kn}_${pat}_$rep.log) $(grep -o '"restored": [a-z]*' $D/k${kn}_${pat}_$rep.log)"
  done; done
  for mm in 18 20; do
    RS_PS8_M8MODE=$mm timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 t32info one_pattern_generic > $D/g${mm}_$rep.log 2>&1 || exit 1
    echo "generic m8_mode $mm $(grep -o '"ms": [0-9.]*' $D/g${mm}_$rep.log)"
  done
done
