set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step issue_bench 100 ./scripts/ubench/issue_bench || exit 1
step pytest_gpu 900 python -m pytest tests/test_gpu.py -x -q -m gpu -k "idx or not (table or mask or jit)"; [ $? -le 1 ] || exit 1
step bench_host 300 python scripts/bench_host.py || exit 1
step traffic 700 bash scripts/gpu_traffic.sh
exit $?
