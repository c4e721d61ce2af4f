#!/bin/bash
# One-table V = 1 step (gen_asm.py v1h) on the per-stripe GF(256) solve: route 2, solve kernel 0 (two
# tables) vs 3 / 4 / 5 (one table; inputs converted 1 / 2 / 4 per LDS round trip), t32info and rand,
# alternating twice; then PMC pass 1-2 of scripts/gpu_r4_ps8_pmc.sh for kernels 0 and 4.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/${PS8:-v1h}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "decode_batch_syndrome_route" > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
for rep in 1 2; do for kn in 0 3 4 5; do for pat in t32info rand; do
  RS_PS8_KERNEL=$kn timeout -k 10 300 python3 -u scripts/bench_patterns.py 4096 $pat device_plans_syndrome > $D/k${kn}_${pat}_$rep.log 2>&1 || exit 1
  echo "kernel $kn $pat $(grep -o '"ms": [0-9.]*' $D/k${kn}_${pat}_$rep.log)"
done; done; done
for kn in 0 4; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
             "SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    RS_PS8_KERNEL=$kn timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $D/pmc_k$kn/p$i -o run -- python3 scripts/bench_patterns.py 4096 t32info device_plans_syndrome > $D/pmc_k${kn}_p$i.log 2>&1
    rc=$?; echo "kernel $kn pass $i rc=$rc"
    case $rc in 0) ;; *) tail -3 $D/pmc_k${kn}_p$i.log; exit $rc;; esac
  done
  echo "== kernel $kn"; python3 scripts/pmc_summary.py $D/pmc_k$kn "k_apply_m8_v1<"
done
