#!/bin/bash
# Round-3 closing set: GPU suite, smoke, the default bench (C3) and its rocprofv3 kernel summary, the C5
# rocprofv3 kernel summary, and the bench under torchrun at world size 1 (RCCL process group).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/z_suite.log 2>&1 || { tail -30 gpurun_out/z_suite.log; exit 1; }
tail -1 gpurun_out/z_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z_smoke.log 2>&1 || { tail -5 gpurun_out/z_smoke.log; exit 1; }
tail -1 gpurun_out/z_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/z_bench_c3.log 2>&1 || { tail -5 gpurun_out/z_bench_c3.log; exit 1; }
tail -1 gpurun_out/z_bench_c3.log | cut -c1-300
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z_prof_c3 -o run -- python3 bench.py > gpurun_out/z_prof_c3.log 2>&1 || exit 1
tail -1 gpurun_out/z_prof_c3.log | cut -c1-300
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z_prof_c5 -o run -- python3 bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 10 > gpurun_out/z_prof_c5.log 2>&1 || exit 1
tail -1 gpurun_out/z_prof_c5.log | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 --cpu-seconds 2 > gpurun_out/z_bench_torchrun1.log 2>&1 || { tail -5 gpurun_out/z_bench_torchrun1.log; exit 1; }
grep '^{' gpurun_out/z_bench_torchrun1.log | tail -1 | cut -c1-300
