set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RS_XJ_SHARE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "jit or xor or shapes or golden" > gpurun_out/pt45.log 2>&1 || { tail -20 gpurun_out/pt45.log; exit 1; }
tail -1 gpurun_out/pt45.log
bash scripts/xj_sweep.sh scripts/sessions/xj_sweep10.txt
