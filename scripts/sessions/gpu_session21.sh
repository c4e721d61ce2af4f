# LDS-table finish (RS_XJ_FIN=1): parity of every xj kernel path with it forced on, then C3 / C2 bench
# against the VALU finish.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
export RS_XJ_FIN=1
step pytest_fin1 600 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "jit or xor or batch or golden" || exit 1
step bench_c3_fin1 300 python bench.py --no-cpu --steps 10 || exit 1
step bench_c2_fin1 300 python bench.py --no-cpu --steps 10 --k 10 --r 4 --symbol 4096 --stripes 262144 || exit 1
export RS_XJ_FIN=0
step bench_c3_fin0 300 python bench.py --no-cpu --steps 10 || exit 1
exit 0
