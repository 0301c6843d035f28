#!/bin/bash
# Round 5 batch 17: stream-ordered ops spin briefly on their readiness event before the sleeping poll: the
# stream-ordered / DDP GPU tests, then the per-process Python latency (blocking / async / ready), twice.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b17}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
log pytest
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -rfE -m gpu \
  tests/test_gpu_allreduce.py tests/test_ddp_overlap.py -k "stream or producer or ddp or overlap" > $OUT/pytest.log 2>&1
rc=$?; log "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  log "py_latency $i"
  GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python benchmarks/py_latency.py --peers 8 --iters 200 --sizes 1048576 \
    > $OUT/py_latency_$i.json 2> $OUT/py_latency_$i.err
  log "rc=$?"
done
log done
exit $rc
