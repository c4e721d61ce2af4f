set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E '^\{|passed|failed' "gpurun_out/$name.log" | cut -c1-400; return $rc; }
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step bench_v1 300 python bench.py --no-cpu --steps 5 --warmup 2 --kernel v1 || exit 1
step bench_patterns 600 python scripts/bench_patterns.py 4096 t32info || exit 1
exit 0
