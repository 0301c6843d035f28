#!/bin/bash
# Round 5 batch 10: config 3 uint8, receive slots of the quantized ring's small steps (PCCL_QUANT_SMALL_SLOTS 3 = the
# round-4 ring, 6, 8) at 32 / 64 ops in flight, interleaved, two passes; then one traced run with the default.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b10}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
POOL=${POOL:-16}
for pass in 1 2; do
  for cq in ${CQS:-32 64}; do
    for sl in ${SLOTS:-3 6 8}; do
      name=p${pass}_cq${cq}_sl$sl
      log "$name"
      PCCL_QUANT_SMALL_SLOTS=$sl timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool $POOL \
        --concurrent 8 --stripes 4 --concurrent-quant $cq --repeat 2 --formats uint8 > $OUT/$name.json 2> $OUT/$name.err
      rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
log "trace"
PCCL_TRACE_OPS=1 timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool $POOL --concurrent 8 \
  --stripes 4 --concurrent-quant 32 --repeat 2 --formats uint8 --log-dir $OUT/logs_cq32 > $OUT/trace_cq32.json \
  2> $OUT/trace_cq32.err
log "rc=$?"
log done
