# Sweep of bit-plane XOR kernel generation knobs on the bench config (encode + decode).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/xj_sweep.jsonl
: > $OUT
while read -r cfg; do
  [ -z "$cfg" ] && continue
  echo "== $cfg $(date +%T)"
  env $cfg timeout -k 10 180 python3 bench.py --no-cpu --steps 5 --warmup 2 --kernel jit > gpurun_out/sw.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "rc=$rc"; tail -5 gpurun_out/sw.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sw.log').read().strip().splitlines()[-1]); print(json.dumps({'cfg': sys.argv[1], 'value': d['value'], 'enc_ms': d['encode_ms'], 'dec_ms': d['decode_ms'], 'parity': d['parity']}))" "$cfg" | tee -a $OUT
done < "${1:-scripts/xj_sweep.txt}"
