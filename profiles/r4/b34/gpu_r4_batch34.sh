#!/bin/bash
# Round 4 batch 34: quantized ring frames and all-gather forwarding granularity below the 16 MiB piece
# (PCCL_QUANT_AG_GRAN = 16 / 8 / 4 MiB of quantized bytes), interleaved; the all-gather's per-hop latency is one
# frame crossing the loopback TCP stripe.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b34
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
timeout -k 10 500 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 6 --ops 3 \
  --variants "g16:PCCL_QUANT_AG_GRAN=16777216;g8:PCCL_QUANT_AG_GRAN=8388608;g4:PCCL_QUANT_AG_GRAN=4194304" \
  > $OUT/gran.jsonl 2> $OUT/gran.err || exit 1
cat $OUT/gran.jsonl
exit 0
