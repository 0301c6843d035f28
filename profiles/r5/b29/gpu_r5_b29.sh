#!/bin/bash
# Round 5 batch 29: config 3 uint8 with the per-op size fixed (64 MiB fp32 per op, the bench's op at 2 GiB / 32) and
# the number of ops growing: 1 / 4 / 8 / 32 ops in flight (pool 16, 4 stripes, 512 KiB); one op alone shows the
# per-step chain (latency + own processing), more ops the cost of sharing the connections.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b29}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for cfg in 64:1 256:4 512:8 2048:32 64:1 2048:32; do
  IFS=: read mib cq <<< "$cfg"
  name=mib${mib}_cq${cq}_$(date +%s)
  log "$name"
  timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib $mib --pool 16 --concurrent 8 --stripes 4 \
    --stripe-min-kib 512 --concurrent-quant $cq --repeat 3 --formats uint8 > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
log done
