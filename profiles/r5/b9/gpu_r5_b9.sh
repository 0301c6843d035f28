#!/bin/bash
# Round 5 batch 9: config 3 connection-pool sweep with the per-op connection groups: uint8 at 32 / 64 ops in flight
# over pools of 16 / 24 / 32 connections per neighbour (1 Gbit/s flows, 25 Gbit/s links), fp32 at 8 ops.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b9}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pool in ${POOLS:-24 32 16}; do
  for cq in ${CQS:-32 64}; do
    name=p${pool}_cq$cq
    log "$name"
    timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool $pool --concurrent 8 --stripes 4 \
      --concurrent-quant $cq --repeat 2 --formats ${FORMATS:-fp32,uint8} > $OUT/$name.json 2> $OUT/$name.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log done
