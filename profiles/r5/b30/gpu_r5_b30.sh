#!/bin/bash
# Round 5 batch 30: one quantized op alone over the WAN relay (64 MiB fp32 -> uint8, 8 peers), traced per step:
# 4 stripes of >= 512 KiB vs 8 of >= 256 KiB.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b30}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for cfg in 4:512 8:256; do
  IFS=: read st smin <<< "$cfg"
  name=s${st}_m$smin
  log "$name"
  PCCL_TRACE_OPS=1 timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 64 --pool 16 --concurrent 8 \
    --stripes $st --stripe-min-kib $smin --concurrent-quant 1 --repeat 3 --formats uint8 --log-dir $OUT/logs_$name \
    > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python profiles/scripts_archive/quant_trace_breakdown.py $OUT/logs_$name/peer0.err --last-ops 2 > $OUT/breakdown_$name.md 2>&1
done
log done
