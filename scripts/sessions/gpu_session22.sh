# Device-built per-stripe decode plans: parity (per-stripe tests, tail fix), then the many-patterns bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
step pytest_batch 600 python -u -m pytest tests/test_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "decode_batch or golden or tail" || exit 1
step bench_patterns 600 python scripts/bench_patterns.py 4096 t32info || exit 1
step bench_patterns_rand 600 python scripts/bench_patterns.py 4096 rand || exit 1
exit 0
