set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E '^\{|passed|failed|Error' "gpurun_out/$name.log" | cut -c1-200; return $rc; }
step pytest_m16 600 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "m16 or c5_ or wide_r or large_n or max_n or gmat" || exit 1
step bench_c5_asm 600 python bench.py --no-cpu --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 1024 || exit 1
grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench_c5_asm.log
exit 0
