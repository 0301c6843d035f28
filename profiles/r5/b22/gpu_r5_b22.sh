#!/bin/bash
# Round 5 batch 22: config 3 uint8 with wider connection groups on larger pools (pool / stripes / stripe minimum KiB /
# ops in flight), against the bench's setting 16 / 4 / 512 / 32; two passes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b22}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for cfg in ${CFGS:-16:4:512:32 32:8:256:32 24:6:256:32 32:8:256:64 32:4:512:32}; do
    IFS=: read pool st smin cq <<< "$cfg"
    name=p${pass}_pool${pool}_s${st}_m${smin}_cq$cq
    log "$name"
    timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool $pool --concurrent 8 --stripes $st \
      --stripe-min-kib $smin --concurrent-quant $cq --repeat 2 --formats uint8 > $OUT/$name.json 2> $OUT/$name.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log done
