#!/bin/bash
# Round 5 batch 34: config 5 with the master's peer exit watcher vs PCCL_PEER_EXIT_WATCH=0 (TCP and xGMI), then the
# GPU fault-tolerance and stress tests with the watcher on.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b34}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for k in 1 2; do
  for t in tcp ipc; do
    for w in 1 0; do
      log "ft $k $t watch=$w"
      PCCL_PEER_EXIT_WATCH=$w timeout -k 10 200 python -u benchmarks/fault_tolerance.py --transport $t \
        > $OUT/ft_${t}_w${w}_$k.json 2> $OUT/ft_${t}_w${w}_$k.err
      rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
log pytest
timeout -k 10 700 python -u -m pytest tests/test_fault_tolerance.py tests/test_stress.py tests/test_benchmarks.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; log "pytest rc=$rc"
