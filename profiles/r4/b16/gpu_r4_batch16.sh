#!/bin/bash
# Round 4 batch 16: quantized ring piece size again with the fused quantize + owner-parity kernel (16 / 32 / 64 MiB,
# interleaved), then a rocprofv3 kernel + copy trace of the default quantized ring (per-kernel stats for profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=gpurun_out/r4_b16
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 6 --ops 3 \
  --variants "p16:PCCL_QUANT_PIECE_BYTES=16777216;p32:PCCL_QUANT_PIECE_BYTES=33554432;p64:PCCL_QUANT_PIECE_BYTES=67108864" \
  > $OUT/pieces.jsonl 2> $OUT/pieces.err || exit 1
cat $OUT/pieces.jsonl
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
  --output-format csv -d $ROOT/$OUT/quant -o run -- python3 $ROOT/scripts/ring_ab_interleaved.py --quant --pool 2 \
  --windows 1 --ops 3 --warmup 2 --variants "base:" > $ROOT/$OUT/quant.log 2>&1) || { tail -20 $OUT/quant.log; exit 1; }
python3 scripts/copy_timeline.py $OUT/quant 10 > $OUT/quant.timeline.md
rm -f $OUT/quant/*/*/*kernel_trace.csv $OUT/quant/*/*/*memory_copy_trace.csv 2>/dev/null
find $OUT/quant -name "*stats.csv" | head
exit 0
