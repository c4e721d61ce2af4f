set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
ok() { [ "$1" -le 1 ]; }
step pytest_gpu 900 python -m pytest tests/test_gpu.py -x -q -m gpu -k "idx or not (table or mask or jit)"; ok $? || exit 1
step bench_idx 600 python bench.py --no-cpu; ok $? || exit 1
step pmc_sq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq3 -o bench -- python3 bench.py --stripes 1024 --steps 2 --warmup 1 --no-cpu --profile-only
exit $?
