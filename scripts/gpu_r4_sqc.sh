#!/bin/bash
# Scalar-cache behaviour of the V = 1 kernel: per-stripe solve (every stripe its own records) vs one shared
# pattern (records shared by every block): SQC_DCACHE_* and SMEM counts in one PMC pass each.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${PS8:-sqc}
mkdir -p $D
C="SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $C -d $D/ps -o run -- python3 scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/ps.log 2>&1 || { tail -3 $D/ps.log; exit 1; }
RS_PS8_M8MODE=18 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $C -d $D/one -o run -- python3 scripts/bench_patterns.py 4096 t32info one_pattern_generic > $D/one.log 2>&1 || { tail -3 $D/one.log; exit 1; }
echo "== per-stripe"; python3 scripts/pmc_summary.py $D/ps "k_apply_m8_v1<"
echo "== one pattern"; python3 scripts/pmc_summary.py $D/one "k_apply_m8_v1<"
