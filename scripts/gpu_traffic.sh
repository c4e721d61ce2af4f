# HBM traffic of the dominant bench kernel: two separate --pmc passes, then scripts/traffic.py.
# usage: gpu_traffic.sh KERNEL_SUBSTR BENCH_KERNEL_NAME
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d gpurun_out/tr_fetch -o run -- python3 bench.py --profile-only --steps 2 --warmup 1 > gpurun_out/tr_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d gpurun_out/tr_write -o run -- python3 bench.py --profile-only --steps 2 --warmup 1 > gpurun_out/tr_write.log 2>&1 || exit $?
python3 scripts/traffic.py gpurun_out/tr_fetch gpurun_out/tr_write "$1" k128_r32_S65536_n8192_t32 "$2" > gpurun_out/traffic.json
