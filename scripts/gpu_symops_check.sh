set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
D=gpurun_out/symE; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "symbol_ops" --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?; tail -2 $D/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $D/pytest.log | head -20; exit $rc; }
timeout -k 10 200 python3 -u scripts/fuzz_parity.py 8088 120 symops > $D/fuzz.log 2>&1 || { tail -5 $D/fuzz.log; exit 1; }
tail -1 $D/fuzz.log
timeout -k 10 120 python -u scripts/bench_symbol_ops.py > $D/bench.log 2>&1 || exit 1
grep '^{' $D/bench.log | cut -c1-160
