#!/bin/bash
# Round 4 batch 35: quantized ring stripes per neighbour with the final copies (pool 4; PCCL_RING_STRIPES 2 / 3 / 4,
# interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b35
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
timeout -k 10 500 python -u scripts/ring_ab_interleaved.py --quant --pool 4 --windows 6 --ops 3 \
  --variants "s2:PCCL_RING_STRIPES=2;s3:PCCL_RING_STRIPES=3;s4:PCCL_RING_STRIPES=4" > $OUT/stripes.jsonl 2> $OUT/stripes.err || exit 1
cat $OUT/stripes.jsonl
exit 0
