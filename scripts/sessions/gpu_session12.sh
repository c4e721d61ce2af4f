set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step pytest_gpu 1000 python -m pytest tests/test_gpu.py -x -q -m gpu; [ $? -le 1 ] || exit 1
step bench_auto 600 python bench.py --no-cpu || exit 1
step bench_v1 600 python bench.py --no-cpu --kernel v1
exit $?
