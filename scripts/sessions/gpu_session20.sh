set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
step pytest_gpu 900 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step bench_host 600 python scripts/bench_host.py
exit 0
