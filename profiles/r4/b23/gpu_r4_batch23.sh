#!/bin/bash
# Round 4 batch 23: the reduce-scatter's host->device copies are the bottleneck of both device rings (one shared
# copy-engine queue, ~45 GB/s; profiles/r4/b22 per-step trace). A/B: every k-th received piece copied on the peer's
# own op stream instead (PCCL_RS_H2D_SPLIT=k; 0 = all on the shared queue, 1 = all on the op stream), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b23
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --pool 2 --windows 4 --ops 4 \
  --variants "s0:PCCL_RS_H2D_SPLIT=0;s2:PCCL_RS_H2D_SPLIT=2;s1:PCCL_RS_H2D_SPLIT=1;s3:PCCL_RS_H2D_SPLIT=3" \
  > $OUT/ring.jsonl 2> $OUT/ring.err || exit 1
cat $OUT/ring.jsonl
timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 4 --ops 3 \
  --variants "s0:PCCL_RS_H2D_SPLIT=0;s2:PCCL_RS_H2D_SPLIT=2;s1:PCCL_RS_H2D_SPLIT=1" \
  > $OUT/quant.jsonl 2> $OUT/quant.err || exit 1
cat $OUT/quant.jsonl
exit 0
