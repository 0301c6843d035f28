#!/bin/bash
# Round 5 batch 16: the DDP-overlap GPU tests (a SIGSEGV in the full run r5_full2) with native backtraces on fatal
# signals (PCCL_DEBUG_BACKTRACE_SIGNAL=1), twice, then the rest of the GPU suite from there on if they pass.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b16}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DEBUG_BACKTRACE_SIGNAL=1
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for i in 1 2; do
  log "ddp_overlap $i"
  timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -rfE -m gpu \
    tests/test_ddp_overlap.py > $OUT/ddp_overlap_$i.log 2>&1
  rc=$?; log "rc=$rc"; [ $rc -le 1 ] || exit $rc
done
log done
