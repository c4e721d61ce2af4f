set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"; return $rc; }
step bench_c2 300 python bench.py --k 10 --r 4 --symbol 4096 --stripes 1024 --no-cpu --steps 20
step bench_c2_big 300 python bench.py --k 10 --r 4 --symbol 4096 --stripes 262144 --no-cpu --steps 10
step bench_c5 600 python bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --no-cpu --steps 2 --warmup 1
step bench_host 600 python scripts/bench_host.py
exit 0
