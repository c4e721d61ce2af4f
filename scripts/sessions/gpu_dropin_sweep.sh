#!/bin/bash
# Per-call arena path knobs at the C3 shape: column chunks x repair write-back (DMA / k_put_rows) x
# zero-copy launches (the XOR kernel streams the page-locked arena across PCIe).
set -o pipefail
mkdir -p gpurun_out
for cfg in "2 1 1" "2 1 0" "1 0 0" "4 0 0"; do
    set -- $cfg
    echo -n "chunks=$1 put=$2 zc=$3 " | tee -a gpurun_out/dropin_sweep.log
    RS_AMD_DROPIN_CHUNKS=$1 RS_AMD_DROPIN_PUT=$2 RS_AMD_DROPIN_ZC=$3 timeout -k 10 60 ./scripts/bench_dropin 128 32 65536 64 \
        | tee -a gpurun_out/dropin_sweep.log || exit 1
done
