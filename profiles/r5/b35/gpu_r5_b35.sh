#!/bin/bash
# Round 5 batch 35: config 4 over TCP (1B fp32 late joiner) with the outdated keys fetched over 1 / 4 / 8 parallel
# connections (PCCL_SS_STREAMS), interleaved over two passes; then the GPU shared-state tests.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b35}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for k in 1 4 8; do
    log "pass $pass streams $k"
    PCCL_SS_STREAMS=$k timeout -k 10 200 python -u benchmarks/shared_state_sync.py --transport tcp --params 1e9 \
      > $OUT/c4_p${pass}_s$k.json 2> $OUT/c4_p${pass}_s$k.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "shared_state or late_joiner or sync_shared or checkpoint or diloco" > $OUT/pytest.log 2>&1
rc=$?; log "pytest rc=$rc"
