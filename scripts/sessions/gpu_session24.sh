# m = 16 hand-scheduled kernel: parity, then C5 (k=4096, r=1024, 1 KiB, 1024 stripes) asm vs compiled.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-900; return $rc; }
step pytest_m16 600 python -u -m pytest tests/test_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "m16 or c5_ or wide_r or large_n or max_n or gmat" || exit 1
step bench_c5_asm 600 python bench.py --no-cpu --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 1024 || exit 1
step bench_c5_compiled 600 python bench.py --no-cpu --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 1024 --kernel m16c || exit 1
exit 0
