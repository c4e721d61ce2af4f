set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep '^{' "gpurun_out/$name.log" | cut -c1-700; return 0; }
step bench_c5_plain 600 python bench.py --no-cpu --profile-only --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 256 --kernel m16p
step bench_c5_asm 600 python bench.py --no-cpu --profile-only --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 256
exit 0
