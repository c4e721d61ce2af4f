# The driver's round-end sequence on the current tree: GPU tests, smoke, default bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E '^\{|passed|failed|smoke' "gpurun_out/$name.log" | cut -c1-600; return $rc; }
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python bench.py || exit 1
exit 0
