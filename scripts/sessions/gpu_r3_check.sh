#!/bin/bash
# Round-3 GPU check: the -m gpu suite, smoke, then the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gputest.log 2>&1 || { tail -30 gpurun_out/r3_gputest.log; exit 1; }
tail -1 gpurun_out/r3_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -5 gpurun_out/r3_smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r3_bench.log 2>&1 || { tail -5 gpurun_out/r3_bench.log; exit 1; }
tail -1 gpurun_out/r3_bench.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 --cpu-seconds 2 > gpurun_out/r3_bench_torchrun1.log 2>&1 || { tail -5 gpurun_out/r3_bench_torchrun1.log; exit 1; }
grep '^{' gpurun_out/r3_bench_torchrun1.log | tail -1 | cut -c1-400
