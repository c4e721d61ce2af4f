#!/bin/bash
# GF(256) per-stripe route and the generic V = 1 step: GPU tests (goldens through every GF(256) variant,
# the per-stripe routes), then scripts/bench_patterns.py A/Bs (4096 C3 stripes; t = 32 information
# erasures and random patterns): solve kernel 0 (two tables) vs 3 (one table) on both fixed passes, the
# one-pattern generic kernel m8_mode 18 vs 20, and a rocprofv3 kernel summary of the one-table solve.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${PS8:-ps8}
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "golden_batch or decode_batch or edge_empty or reenc" > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
for rt in 2 1; do for kn in 0 3; do for pat in t32info rand; do
  RS_PS8_ROUTE=$rt RS_PS8_KERNEL=$kn timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 $pat device_plans_syndrome > $D/r${rt}_k${kn}_$pat.log 2>&1 || exit 1
  echo "route $rt kernel $kn $pat $(grep '^{' $D/r${rt}_k${kn}_$pat.log)"
done; done; done
for mm in 18 20; do
  RS_PS8_M8MODE=$mm timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 t32info one_pattern_generic > $D/gen_m$mm.log 2>&1 || exit 1
  echo "generic m8_mode $mm $(grep '^{' $D/gen_m$mm.log)"
done
RS_PS8_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- \
  python3 -u scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/prof.log 2>&1 || exit 1
python3 - $D/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
