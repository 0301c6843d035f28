#!/bin/bash
# Round 5 batch 12: config 3 uint8, stripe minimum (PCCL_STRIPE_MIN_BYTES, now down to 256 KiB) x ops in flight: how
# many ops share a connection group (groups of op_stripes connections) vs how many connections carry data.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b12}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for cfg in ${CFGS:-32:1024 32:512 64:1024 64:512 64:256 128:512 16:1024}; do
  IFS=: read cq smin <<< "$cfg"
  name=cq${cq}_min${smin}k
  log "$name"
  timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 --concurrent 8 --stripes 4 \
    --stripe-min-kib $smin --concurrent-quant $cq --repeat 2 --formats uint8 > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
log done
