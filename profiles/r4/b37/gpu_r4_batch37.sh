#!/bin/bash
# Round 4 batch 37: quantized ring lane staggering (the second lane starts once the first lane's first payload is
# quantized) on / off with the per-lane copies (PCCL_QUANT_NO_GATE=1: both lanes start at once), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b37
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
timeout -k 10 500 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 6 --ops 3 \
  --variants "gate:PCCL_QUANT_NO_GATE=0;nogate:PCCL_QUANT_NO_GATE=1" > $OUT/gate.jsonl 2> $OUT/gate.err || exit 1
cat $OUT/gate.jsonl
exit 0
