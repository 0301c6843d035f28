#!/bin/bash
# Round 4 batch 29: config 3 (WAN emulator) after the quantized ring's copies moved to the lane streams measured slower
# than before (profiles/r4/wan3 vs wan2). A/B in alternating processes: PCCL_QUANT_SHARED_H2D=1 restores the earlier
# copies (reduce-scatter through the process-wide queue, all-gather de-quantized from pinned memory).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b29
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3; do
  for v in 1 0; do
    PCCL_QUANT_SHARED_H2D=$v timeout -k 10 200 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 \
      --concurrent 8 --stripes 4 --concurrent-quant 32 --formats uint8 > $OUT/wan_old${v}_$rep.json \
      2> $OUT/wan_old${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$OUT/wan_old${v}_$rep.json')); print('shared_h2d=$v', d['formats']['uint8']['seconds'])"
  done
done
PCCL_DISABLE_IPC=1 timeout -k 10 300 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 4 --ops 3 \
  --variants "new:PCCL_QUANT_SHARED_H2D=0;old:PCCL_QUANT_SHARED_H2D=1" > $OUT/ring.jsonl 2> $OUT/ring.err || exit 1
cat $OUT/ring.jsonl
exit 0
