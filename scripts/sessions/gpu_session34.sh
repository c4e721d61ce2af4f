set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --stripes 1024 --steps 3 --warmup 1 --cpu-seconds 2 > gpurun_out/b34.log 2>&1; rc=$?
grep -o '"cpu_baseline": {[^}]*}\|"parity": "[^"]*"\|"value": [0-9.]*' gpurun_out/b34.log; tail -2 gpurun_out/b34.log | cut -c1-300
exit $rc
