#!/bin/bash
# Round 5 batch 8: config 3 uint8 at 32 and 64 ops in flight with PCCL_TRACE_OPS=1 (per-step marks of every op, with
# the op thread's start on the host-wide clock) and every peer's stderr kept.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b8}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for cq in ${CQS:-32 64}; do
  log "wan trace cq=$cq"
  PCCL_TRACE_OPS=1 timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 --concurrent 8 \
    --stripes 4 --concurrent-quant $cq --repeat 2 --formats uint8 --log-dir $OUT/logs_cq$cq > $OUT/wan_cq$cq.json \
    2> $OUT/wan_cq$cq.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
log done
