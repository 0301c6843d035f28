#!/bin/bash
# Round 5 batch 14: why larger connection pools are slower through the WAN relay: pools 16 / 32 with the peers' CPU
# use (sum of the 8 peer processes' cores while the multi-op runs) and the relay's.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b14}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pool in 16 32 16 32; do
  name=p${pool}_$(date +%s)
  log "$name"
  timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool $pool --concurrent 8 --stripes 4 \
    --concurrent-quant 32 --stripe-min-kib 512 --repeat 2 --formats fp32,uint8 > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
log done
