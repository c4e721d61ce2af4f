set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread; [ $? -le 1 ] || exit 1
step traffic 700 bash scripts/gpu_traffic.sh rs_xj rs_xj || exit 1
cp gpurun_out/traffic.json profiles/traffic.json
step bench_full 600 python bench.py || exit 1
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof17 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu --profile-only
exit $?
