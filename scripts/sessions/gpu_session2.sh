set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
ok() { [ "$1" -le 1 ]; }
step pytest_gpu 900 python -m pytest tests/test_gpu.py -x -q -m gpu -k "idx or not (table or mask or jit)"; ok $? || exit 1
step bench_idx 600 python bench.py; ok $? || exit 1
step prof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_idx -o bench -- python3 bench.py --steps 5 --warmup 1 --no-cpu --profile-only; ok $? || exit 1
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o bench -- python3 bench.py --stripes 2048 --steps 2 --warmup 1 --no-cpu --profile-only; ok $? || exit 1
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o bench -- python3 bench.py --stripes 2048 --steps 2 --warmup 1 --no-cpu --profile-only; ok $? || exit 1
step pmc_sq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_sq -o bench -- python3 bench.py --stripes 1024 --steps 2 --warmup 1 --no-cpu --profile-only
exit $?
