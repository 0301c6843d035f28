#!/bin/bash
# Round 5 batch 36: config 5 (TCP and xGMI) with the round-robin bandwidth-probe schedule: optimize_topology time,
# then the GPU topology / fault-tolerance tests.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b36}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for t in tcp ipc tcp; do
  log "ft $t"
  timeout -k 10 200 python -u benchmarks/fault_tolerance.py --transport $t > $OUT/ft_${t}_$(date +%s).json 2> $OUT/ft_$t.err
  rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
log pytest
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "topology or optimize or fault or stress" > $OUT/pytest.log 2>&1
rc=$?; log "pytest rc=$rc"
