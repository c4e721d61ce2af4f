set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
step bench_c2_big 300 python bench.py --k 10 --r 4 --symbol 4096 --stripes 262144 --no-cpu --steps 10
step bench_c3 300 python bench.py --no-cpu --steps 5
exit 0
