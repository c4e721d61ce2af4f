#!/bin/bash
# Round-4 start: registration-churn probe (no copies into reused ranges), C3 bench on the current tree,
# kernel split of the GF(256) per-stripe syndrome route (t = 32 all-distinct patterns), C5 PMC traffic on
# the current kernels and the C5 kernels' L2 hit / miss split.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r4s
mkdir -p $D
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 -o $D/reg_probe scripts/ubench/reg_probe.hip || exit 1
timeout -k 10 120 $D/reg_probe 40 7 > $D/reg_probe.log 2>&1 || { cat $D/reg_probe.log; exit 1; }
cat $D/reg_probe.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > $D/bench_c3.log 2>&1 || { tail -5 $D/bench_c3.log; exit 1; }
grep '^{' $D/bench_c3.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/ps8 -o run -- \
  python3 -u scripts/bench_patterns.py 4096 t32info device_plans_syndrome,one_pattern_xj > $D/ps8.log 2>&1 || { tail -5 $D/ps8.log; exit 1; }
grep '^{' $D/ps8.log
TR=r4s/c5 bash scripts/gpu_traffic.sh --k 4096 --r 1024 --symbol 1024 --stripes 1024 || exit 1
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCC_REQ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $D/c5tcc$i -o run -- \
    python3 bench.py --profile-only --steps 2 --warmup 3 --k 4096 --r 1024 --symbol 1024 --stripes 1024 > $D/c5tcc$i.log 2>&1 || exit $?
done
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --k 4096 --r 1024 --symbol 1024 --stripes 1024 > $D/bench_c5.log 2>&1 || { tail -5 $D/bench_c5.log; exit 1; }
grep '^{' $D/bench_c5.log | cut -c1-300
