#!/bin/bash
# HBM traffic per launch of the bench's encode and decode kernels: two separate --pmc passes over
# `bench.py --profile-only`, then scripts/traffic.py (records keyed by each leg's exact kernel).
# usage: [TR=name] gpu_traffic.sh [extra bench args]   (output gpurun_out/${TR:-tr}affic.json)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=gpurun_out/${TR:-tr}
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d ${T}_fetch -o run -- python3 bench.py --profile-only --steps 2 --warmup 3 "$@" > ${T}_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d ${T}_write -o run -- python3 bench.py --profile-only --steps 2 --warmup 3 "$@" > ${T}_write.log 2>&1 || exit $?
cfg=$(python3 -c "import json; print([json.loads(x) for x in open('${T}_fetch.log') if x.startswith('{')][-1]['roofline']['traffic_key'])") || exit 1
python3 scripts/traffic.py ${T}_fetch ${T}_write "$cfg" > ${T}affic.json
