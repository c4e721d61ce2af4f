# Full GPU suite + smoke + default bench line after a container rebuild (syndrome route included).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt55.log 2>&1 || { tail -40 gpurun_out/pt55.log; exit 1; }
tail -1 gpurun_out/pt55.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke55.log 2>&1 || { tail -5 gpurun_out/smoke55.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench55.log 2>&1 || { tail -5 gpurun_out/bench55.log; exit 1; }
tail -1 gpurun_out/bench55.log
