#!/bin/bash
# One-pattern syndrome route with overlapped chunks (m16_cs_overlap): route GPU tests, then C5 bench A/B
# (overlap on = default, off via bench.py --opt m16_cs_overlap=0) on the same box.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/cs_overlap
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "cs16 or m16 or golden or decode_batch" > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 10 --warmup 3 --no-cpu > $D/c5_on_$i.log 2>&1 || exit 1
  grep '^{' $D/c5_on_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('on ', d['value'], d['encode_ms'], d['decode_ms'])"
  timeout -k 10 300 python3 -u bench.py --k 4096 --r 1024 --symbol 1024 --stripes 1024 --steps 10 --warmup 3 --no-cpu --opt m16_cs_overlap=0 > $D/c5_off_$i.log 2>&1 || exit 1
  grep '^{' $D/c5_off_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('off', d['value'], d['encode_ms'], d['decode_ms'])"
done
timeout -k 10 300 python3 -u scripts/bench_patterns_c5.py 1024 > $D/patterns.log 2>&1; rc=$?; grep one_pattern $D/patterns.log; exit $rc
