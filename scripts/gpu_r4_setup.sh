#!/bin/bash
# V = 1 kernels with the ring prologue issued before the LDS table copy: GF(256) GPU tests, phase stamps
# (diagnostic library), per-stripe solve (route 2, t32info / rand) and the one-pattern generic kernel.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${PS8:-setup}
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "golden_batch or decode_batch or edge_empty or reenc or drop_in" > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
RS_AMD_LIB=$PWD/reed-solomon_amd/librs_amd_diag.so timeout -k 10 300 python3 -u scripts/gpu_stamps_v1.py > $D/stamps.log 2>&1 || exit 1
grep '^{' $D/stamps.log
for rep in 1 2; do
  for pat in t32info rand; do
    timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 $pat device_plans_syndrome > $D/ps_${pat}_$rep.log 2>&1 || exit 1
    echo "ps $pat $(grep -o '"ms": [0-9.]*' $D/ps_${pat}_$rep.log)"
  done
  for mm in 18 20; do
    RS_PS8_M8MODE=$mm timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 t32info one_pattern_generic > $D/g${mm}_$rep.log 2>&1 || exit 1
    echo "generic m8_mode $mm $(grep -o '"ms": [0-9.]*' $D/g${mm}_$rep.log)"
  done
done
