#!/bin/bash
# Round 5 batch 13: the tests touched since the full run (mixed pool sizes after the per-pool stripe groups, the PCIe
# counter test, wire compatibility, stream-ordered ops), then the per-process Python latency with the idle-stream
# shortcut.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b13}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
log pytest
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -rfE -m gpu \
  tests/test_gpu_allreduce.py tests/test_wire_compat.py -k "mixed_pool or pcie or stream or producer or wire or mixed or staging or striped" \
  > $OUT/pytest.log 2>&1
rc=$?
log "pytest rc=$rc"
tail -n 5 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
log py_latency
GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python benchmarks/py_latency.py --peers 8 --iters 200 --sizes 1048576 \
  > $OUT/py_latency.json 2> $OUT/py_latency.err
log "rc=$?"
log done
exit $rc
