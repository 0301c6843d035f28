#!/bin/bash
# Round 4 batch 8: A/B of the quantized ring's reduce-scatter input (copy engine -> HBM vs kernels reading pinned
# memory, temporary PCCL_TMP_QRS_PINNED) and of the 2-peer ring's stripes per step (PCCL_RING_STRIPES 4 / 8).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b8
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
AB="python -u scripts/ring_ab_interleaved.py"
timeout -k 10 300 $AB --quant --pool 2 --windows 4 --ops 3 \
  --variants "staged:PCCL_TMP_QRS_PINNED=0;pinned:PCCL_TMP_QRS_PINNED=1" > $OUT/q_rs.jsonl 2> $OUT/q_rs.err || exit 1
cat $OUT/q_rs.jsonl
timeout -k 10 300 $AB --peers 2 --pool 8 --windows 4 --ops 5 \
  --variants "s4:PCCL_RING_STRIPES=4;s8:PCCL_RING_STRIPES=8" > $OUT/two_stripes.jsonl 2> $OUT/two_stripes.err || exit 1
cat $OUT/two_stripes.jsonl
timeout -k 10 300 $AB --peers 4 --pool 4 --windows 4 --ops 4 \
  --variants "s4:PCCL_RING_STRIPES=4;s2:PCCL_RING_STRIPES=2" > $OUT/four_stripes.jsonl 2> $OUT/four_stripes.err || exit 1
cat $OUT/four_stripes.jsonl
exit 0
