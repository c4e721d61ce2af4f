set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread; [ $? -le 1 ] || exit 1
step bench_full 600 python bench.py || exit 1
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof14 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --profile-only
exit $?
