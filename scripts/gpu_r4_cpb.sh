#!/bin/bash
# Per-stripe GF(256) solve with several 1 KiB column chunks per workgroup (option m8_ps_cpb, k_apply_m8_v1<6>):
# its GPU tests, then route 2 t32info / rand at cpb 1 / 2 / 4 / 8 / 16, two alternating reps.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${PS8:-cpb}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "decode_batch_syndrome_route or golden_batch" > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
for rep in 1 2; do for cpb in 1 2 4 8 16; do for pat in t32info rand; do
  RS_PS8_CPB=$cpb timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 $pat device_plans_syndrome > $D/c${cpb}_${pat}_$rep.log 2>&1 || exit 1
  echo "cpb $cpb $pat $(grep -o '"ms": [0-9.]*' $D/c${cpb}_${pat}_$rep.log) $(grep -o '"restored": [a-z]*' $D/c${cpb}_${pat}_$rep.log)"
done; done; done
