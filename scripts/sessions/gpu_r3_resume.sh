#!/bin/bash
# Round-3 resume check after the registered-symbol allocator change: GPU suite, smoke, default bench,
# then the mixed fuzz (orbit + per-stripe GF(2^16) + registered drop-in) that faulted before the change.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rs_suite.log 2>&1 || { tail -30 gpurun_out/rs_suite.log; exit 1; }
tail -1 gpurun_out/rs_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rs_smoke.log 2>&1 || { tail -5 gpurun_out/rs_smoke.log; exit 1; }
tail -1 gpurun_out/rs_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/rs_bench.log 2>&1 || { tail -5 gpurun_out/rs_bench.log; exit 1; }
tail -1 gpurun_out/rs_bench.log | cut -c1-300
timeout -k 10 150 python -u scripts/diag_family.py orbit,ps16,dropin_reg 120 3033 > gpurun_out/rs_diag_mix.log 2>&1 || { tail -20 gpurun_out/rs_diag_mix.log; exit 1; }
tail -1 gpurun_out/rs_diag_mix.log
# threaded-block k_cs16 step candidate vs today's gpr-indexed step (scripts/ubench/gen_thread.py)
timeout -k 10 90 ./scripts/ubench/bin/thread_bench > gpurun_out/rs_thread_bench.log 2>&1 || { cat gpurun_out/rs_thread_bench.log; exit 1; }
cat gpurun_out/rs_thread_bench.log
