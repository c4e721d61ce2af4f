set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for th in 4 8 12 16; do
  RS_AMD_HOST_THREADS=$th timeout -k 10 120 ./scripts/bench_dropin 128 32 65536 32 | sed "s/^/threads=$th /" || exit 1
done
