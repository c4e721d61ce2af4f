set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  return $rc
}
step env 300 python -c "import torch;print(torch.__version__, torch.cuda.get_device_name(0), torch.cuda.mem_get_info())" || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; [ $rc -le 1 ] || exit $rc
step pytest_gpu 900 python -m pytest tests/test_gpu.py -x -q -m gpu; rc=$?; [ $rc -le 1 ] || exit $rc
step bench_small 300 python bench.py --stripes 512 --steps 3 --warmup 1 --cpu-stripes 8 ; rc=$?; [ $rc -le 1 ] || exit $rc
step bench_table 300 python bench.py --stripes 2048 --steps 3 --warmup 1 --kernel table --no-cpu ; rc=$?; [ $rc -le 1 ] || exit $rc
step bench_mask 300 python bench.py --stripes 2048 --steps 3 --warmup 1 --kernel mask --no-cpu ; rc=$?; [ $rc -le 1 ] || exit $rc
step bench_full 600 python bench.py ; rc=$?
exit $rc
