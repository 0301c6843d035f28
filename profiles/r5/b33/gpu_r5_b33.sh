#!/bin/bash
# Round 5 batch 33: config 5 over TCP and xGMI with the victim's reap time (kill -> its process gone).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b33}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for t in tcp ipc tcp; do
  log "ft $t"
  timeout -k 10 200 python -u benchmarks/fault_tolerance.py --transport $t > $OUT/ft_${t}_$(date +%s).json 2> $OUT/ft_$t.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
log done
