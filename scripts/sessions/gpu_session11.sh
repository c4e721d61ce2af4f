set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step issue_bench2 150 ./scripts/ubench/issue_bench || exit 1
step bench_host 300 python scripts/bench_host.py || exit 1
step bench_full 600 python bench.py
exit $?
