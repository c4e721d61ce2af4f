#!/bin/bash
# k_cs16t (4 cosets, one-asm loop): GPU suite, C5 A/B (default vs m16_cs_thread=0), C5 PMC traffic of both
# legs, C5 per-stripe patterns, then route-family fuzz on the new default.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c_suite.log 2>&1 || { tail -30 gpurun_out/c_suite.log; exit 1; }
tail -1 gpurun_out/c_suite.log
for thr in 1 0; do
timeout -k 10 300 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 20 --no-cpu --opt m16_cs_thread=$thr > gpurun_out/c_c5_$thr.log 2>&1 || { tail -5 gpurun_out/c_c5_$thr.log; exit 1; }
echo "thr=$thr"; tail -1 gpurun_out/c_c5_$thr.log | cut -c1-200
done
TR=c5tr bash scripts/gpu_traffic.sh --k 4096 --r 1024 --symbol 1024 --stripes 1024 || exit 1
cat gpurun_out/c5traffic.json | head -30
timeout -k 10 300 python -u scripts/bench_patterns_c5.py 1024 > gpurun_out/c_patterns_c5.log 2>&1 || { tail -5 gpurun_out/c_patterns_c5.log; exit 1; }
head -2 gpurun_out/c_patterns_c5.log
timeout -k 10 300 python -u scripts/fuzz_parity.py 3041 240 route,reenc,ps16,orbit,m16 > gpurun_out/c_fuzz.jsonl 2>&1 || { tail -5 gpurun_out/c_fuzz.jsonl; exit 1; }
tail -1 gpurun_out/c_fuzz.jsonl
