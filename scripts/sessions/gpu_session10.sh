set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step pytest_gpu 900 python -m pytest tests/test_gpu.py -x -q -m gpu -k "idx or not (table or mask or jit)"; [ $? -le 1 ] || exit 1
step ablate 600 python scripts/gpu_ablate.py 2048 || exit 1
grep variant gpurun_out/ablate.log
step bench_idx 600 python bench.py --no-cpu
exit $?
