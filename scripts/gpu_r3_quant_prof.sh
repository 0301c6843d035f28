#!/bin/bash
# Round 3: quantized device ring (uint8 min-max, 8 peers x 1 GiB): interleaved A/B of the fused min / max
# (PCCL_QUANT_FUSED_MINMAX) and a rocprofv3 kernel-stats profile of the same run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${OUTDIR:-r3_quant}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
timeout -k 10 300 python -u scripts/ring_ab_interleaved.py --quant --windows ${WINDOWS:-6} --ops 4 \
  --variants "fused:PCCL_QUANT_FUSED_MINMAX=1;pass:PCCL_QUANT_FUSED_MINMAX=0" > $OUT/ab.jsonl 2> $OUT/ab.err \
  || { tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o quant -- \
  python3 "$R/scripts/ring_ab_interleaved.py" --quant --windows 2 --ops 3 --variants "fused:PCCL_QUANT_FUSED_MINMAX=1" \
  > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
