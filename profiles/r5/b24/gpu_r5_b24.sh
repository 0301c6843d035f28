#!/bin/bash
# Round 5 batch 24: config 3 uint8 with ops launched in K staggered cohorts (cohort k starts k x D ms later; 32 ops in
# flight in total, the bench's pool 16 / 4 stripes / 512 KiB), two interleaved passes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b24}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for cfg in ${CFGS:-1:0 8:6 8:12 16:3 32:1.5 32:3}; do
    IFS=: read k d <<< "$cfg"
    name=p${pass}_k${k}_d$d
    log "$name"
    timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 --concurrent 8 --stripes 4 \
      --stripe-min-kib 512 --concurrent-quant 32 --repeat 2 --formats uint8 --cohorts $k --cohort-delay-ms $d \
      > $OUT/$name.json 2> $OUT/$name.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log done
