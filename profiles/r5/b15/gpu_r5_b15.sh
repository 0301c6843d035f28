#!/bin/bash
# Round 5 batch 15 (experiment): config 3 uint8, 32 ops in flight split into K out-of-phase cohorts (each its own
# multi-op call, cohort k started k x D ms later) vs one multi-op call: does overlapping one cohort's transfers with
# another's latency beat the ~85 ms ring step of ops in step with each other?
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b15}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for cfg in ${CFGS:-1:0 2:30 2:45 4:15 4:22 1:0 2:40}; do
  IFS=: read k d <<< "$cfg"
  name=k${k}_d${d}_$(date +%s)
  log "$name"
  timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 --concurrent 8 --stripes 4 \
    --concurrent-quant 32 --stripe-min-kib 512 --repeat 2 --formats uint8 --cohorts $k --cohort-delay-ms $d \
    > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
log done
