#!/bin/bash
# Kernel breakdown of the C5 per-stripe syndrome route (scripts/prof_ps16.py, 1024 stripes): rocprofv3
# kernel trace + stats, and the wall time of each run.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/ps16_prof
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 -u scripts/prof_ps16.py 1024 > $D/run.log 2>&1
rc=$?; echo "rc=$rc"; cat $D/run.log
exit $rc
