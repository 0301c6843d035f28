#!/bin/bash
# Round 5 batch 28: the staging reserve GPU test, then config 5 over TCP with the reserve next to connect() and the
# tensor created before it, vs --no-reserve, interleaved (two each).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b28}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
log pytest
timeout -k 10 300 python -u -m pytest tests/test_gpu_allreduce.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "reserved_staging or pcie_bytes" > $OUT/pytest.log 2>&1
rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
for k in ${PAIRS:-1 2}; do
  for v in reserve noreserve; do
    log "ft $k $v"
    extra=""; [ $v = noreserve ] && extra="--no-reserve"
    timeout -k 10 200 python -u benchmarks/fault_tolerance.py --transport tcp $extra > $OUT/ft_${v}_$k.json 2> $OUT/ft_${v}_$k.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log done
