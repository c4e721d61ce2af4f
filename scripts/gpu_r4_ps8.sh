#!/bin/bash
# GF(256) per-stripe route: its GPU tests, then scripts/bench_patterns.py (t = 32 information erasures and
# random patterns, 4096 C3 stripes) for the fixed pass (syndromes / re-encode), the overlap and the solve
# kernel, and a rocprofv3 kernel summary of the defaults.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${PS8:-ps8}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "decode_batch or golden_batch or edge_empty or reenc" > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 t32info device_plans_syndrome,one_pattern_xj > $D/t32info.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 rand device_plans_syndrome > $D/rand.log 2>&1 || exit 1
for rt in 1 2; do for ov in 0 1; do for pat in t32info rand; do
  RS_PS8_ROUTE=$rt RS_PS8_OVERLAP=$ov timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 $pat device_plans_syndrome > $D/r${rt}_o${ov}_$pat.log 2>&1 || exit 1
  echo "route $rt overlap $ov $pat $(grep '^{' $D/r${rt}_o${ov}_$pat.log)"
done; done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- \
  python3 -u scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/prof.log 2>&1 || exit 1
for f in t32info rand; do echo "$f $(grep '^{' $D/$f.log)"; done
