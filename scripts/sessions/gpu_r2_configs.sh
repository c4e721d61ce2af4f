#!/bin/bash
# Round-2 lines for the other configurations: C2 (k=10 r=4 4 KiB, the config's 1024 stripes, and 262144
# stripes), C5 (k=4096 r=1024 1 KiB, 1024 stripes) with its rocprofv3 kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
timeout -k 10 300 python bench.py --k 10 --r 4 --symbol 4096 --stripes 1024 --steps 200 > gpurun_out/cfg/c2_1024.log 2>&1 || exit 1
tail -1 gpurun_out/cfg/c2_1024.log | cut -c1-200
timeout -k 10 300 python bench.py --k 10 --r 4 --symbol 4096 --stripes 262144 --steps 40 --no-cpu > gpurun_out/cfg/c2_262144.log 2>&1 || exit 1
tail -1 gpurun_out/cfg/c2_262144.log | cut -c1-200
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg/c5_prof -o run -- python3 bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 10 --warmup 3 --no-cpu > gpurun_out/cfg/c5_prof.log 2>&1 || exit 1
tail -1 gpurun_out/cfg/c5_prof.log | cut -c1-200
