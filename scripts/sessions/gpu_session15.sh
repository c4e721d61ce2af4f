set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest_gpu 900 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread; [ $? -le 1 ] || exit 1
step bench_jit 600 python bench.py --no-cpu --kernel jit || exit 1
step bench_v1jit 600 python bench.py --no-cpu --kernel v1jit --steps 3
exit $?
