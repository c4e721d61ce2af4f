# L1/L2 request counters of the bench's rs_xj encode (does each column's input reach L2 once or twice?)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/pmcl2
mkdir -p $D
i=0
for grp in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_REQ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $D/p$i -o run -- python3 scripts/pmc_xj.py jit 1024 > $D/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) tail -3 $D/p$i.log; exit $rc;; esac
done
exit 0
