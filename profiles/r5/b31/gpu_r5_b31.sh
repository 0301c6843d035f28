#!/bin/bash
# Round 5 batch 31: the 8-process small-op latency matrix with the calls ordered on torch's default (null) stream vs
# a created stream, interleaved, two passes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b31}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for cs in default side; do
    log "pass $pass $cs"
    timeout -k 10 240 python -u benchmarks/py_latency.py --peers 8 --iters 300 --sizes 1048576 --caller-stream $cs \
      > $OUT/lat_p${pass}_$cs.json 2> $OUT/lat_p${pass}_$cs.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log done
