#!/bin/bash
# Round 4 batch 9: the quantized small-chunk hang repro (fixed: a ring ends only when every step's stripes are sent),
# the device-ring edge-case tests, then the batch-8 A/Bs.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b9
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u profiles/scripts_archive/repro_quant_small.py 1 10 > $OUT/repro.log 2>&1 || { tail -5 $OUT/repro.log; exit 1; }
tail -2 $OUT/repro.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "fewer_elements or small_messages or quantized" > $OUT/edge.log 2>&1
rc=$?; tail -3 $OUT/edge.log; [ $rc -le 1 ] || exit $rc
bash profiles/r4/scripts/gpu_r4_batch8.sh
