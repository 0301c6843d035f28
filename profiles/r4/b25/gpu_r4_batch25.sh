#!/bin/bash
# Round 4 batch 25: quantized all-gather consume, kernels reading pinned memory (default) vs host -> HBM on the lane's
# own stream then de-quantize (PCCL_QUANT_AG_STAGED=1), interleaved; then pieces 16 / 32 MiB with the new copies.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b25
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 6 --ops 3 \
  --variants "pinned:PCCL_QUANT_AG_STAGED=0;staged:PCCL_QUANT_AG_STAGED=1" > $OUT/ag.jsonl 2> $OUT/ag.err || exit 1
cat $OUT/ag.jsonl
timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 4 --ops 3 \
  --variants "p32:PCCL_QUANT_PIECE_BYTES=33554432;p16:PCCL_QUANT_PIECE_BYTES=16777216;p64:PCCL_QUANT_PIECE_BYTES=67108864" \
  > $OUT/pieces.jsonl 2> $OUT/pieces.err || exit 1
cat $OUT/pieces.jsonl
exit 0
