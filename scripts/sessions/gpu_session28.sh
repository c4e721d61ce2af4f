set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 env RS_M16_WIDE=1 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread -k "m16" > gpurun_out/pt_wide.log 2>&1; echo "wide tests rc=$? $(tail -1 gpurun_out/pt_wide.log)"
for w in 0 1; do
  timeout -k 10 300 env RS_M16_WIDE=$w python bench.py --no-cpu --steps 2 --warmup 1 --k 4096 --r 1024 --symbol 1024 --stripes 1024 > gpurun_out/c5_w$w.log 2>&1 || exit 1
  echo "wide=$w $(grep -o '"value": [0-9.]*' gpurun_out/c5_w$w.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/c5_w$w.log) $(grep -o '"parity": "[^"]*"' gpurun_out/c5_w$w.log)"
done
exit 0
