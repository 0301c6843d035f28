#!/bin/bash
# Round 4 batch 26: quantized payloads, quantize kernels writing pinned memory directly (default) vs quantize into HBM
# then a device->host copy on a second per-lane stream (PCCL_QUANT_TX_STAGED=1), interleaved; exactness checked by
# the GPU quantized tests under the staged variant.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b26
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
PCCL_QUANT_TX_STAGED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "quant" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
PCCL_DISABLE_IPC=1 timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 6 --ops 3 \
  --variants "pinned:PCCL_QUANT_TX_STAGED=0;staged:PCCL_QUANT_TX_STAGED=1" > $OUT/tx.jsonl 2> $OUT/tx.err || exit 1
cat $OUT/tx.jsonl
exit 0
