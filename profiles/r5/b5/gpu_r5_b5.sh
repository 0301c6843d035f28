#!/bin/bash
# Round 5 batch 5: config 3 (uint8, 50 ms WAN relay) A/B of the connection spread (PCCL_STRIPE_SPREAD=0: round-4
# mapping, 1: lap-shifted) at 16 / 32 / 64 ops in flight, interleaved, two passes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b5}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for cq in 16 32 64; do
    for sp in 0 1; do
      name=p${pass}_cq${cq}_s$sp
      log "$name"
      PCCL_STRIPE_SPREAD=$sp timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 \
        --concurrent 8 --stripes 4 --concurrent-quant $cq --repeat 2 --formats uint8 > $OUT/$name.json 2> $OUT/$name.err
      rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
log done
