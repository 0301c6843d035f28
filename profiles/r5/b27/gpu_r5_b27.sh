#!/bin/bash
# Round 5 batch 27: config 5 over TCP with per-op traces in every peer (the replacement's first op vs steady ops), x2.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b27}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_TRACE_OPS=1
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for k in 1 2; do
  log "ft $k"
  timeout -k 10 200 python -u benchmarks/fault_tolerance.py --transport tcp --log-dir $OUT/ft$k > $OUT/ft$k.json 2> $OUT/ft$k.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
log done
