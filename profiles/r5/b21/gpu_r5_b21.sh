#!/bin/bash
# Round 5 batch 21: per-op stripe groups bounded by the monotone stripe bound: the device-ring GPU tests that stripe
# (uneven chunks with small stripes, mixed pool sizes, striped / staging / wire-compat tests).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b21}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "[$(date +%T)] pytest" >> $OUT/steps.log
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -rfE -m gpu \
  tests/test_gpu_allreduce.py tests/test_wire_compat.py -k "stripe or mixed or device_ring or wire or quantized" \
  > $OUT/pytest.log 2>&1
rc=$?
echo "[$(date +%T)] rc=$rc" >> $OUT/steps.log
tail -n 5 $OUT/pytest.log
exit $rc
