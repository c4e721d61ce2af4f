# rocprof kernel stats for C2 (1024 stripes) and C5 (1024 stripes); HBM traffic of the C5 kernel.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
C5="--k 4096 --r 1024 --symbol 1024 --stripes 1024"
C2="--k 10 --r 4 --symbol 4096 --stripes 1024"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python3 bench.py --no-cpu --profile-only --steps 10 --warmup 3 $C2 > gpurun_out/prof_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --no-cpu --profile-only --steps 2 --warmup 1 $C5 > gpurun_out/prof_c5.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d gpurun_out/c5_fetch -o run -- python3 bench.py --no-cpu --profile-only --steps 1 --warmup 1 $C5 > gpurun_out/c5_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d gpurun_out/c5_write -o run -- python3 bench.py --no-cpu --profile-only --steps 1 --warmup 1 $C5 > gpurun_out/c5_write.log 2>&1 || exit 1
cut -d, -f1-4 gpurun_out/prof_c2/run_kernel_stats.csv | head -4
cut -d, -f1-4 gpurun_out/prof_c5/run_kernel_stats.csv | head -4
