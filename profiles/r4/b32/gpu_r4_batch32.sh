#!/bin/bash
# Round 4 batch 32: rocprofv3 kernel + copy trace of the final quantized ring (8 peers x 1 GiB, uint8; per-lane copies)
# and of the plain ring, summarised per time bin (scripts/copy_timeline.py) with per-kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=gpurun_out/r4_b32
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
for v in quant plain; do
  extra=""; [ $v = quant ] && extra="--quant"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
    --output-format csv -d $ROOT/$OUT/$v -o run -- python3 $ROOT/scripts/ring_ab_interleaved.py $extra --pool 2 \
    --windows 1 --ops 3 --warmup 2 --variants "base:" > $ROOT/$OUT/$v.log 2>&1) || { tail -20 $OUT/$v.log; exit 1; }
  python3 scripts/copy_timeline.py $OUT/$v 10 > $OUT/$v.timeline.md
  rm -f $OUT/$v/run_kernel_trace.csv $OUT/$v/run_memory_copy_trace.csv
done
exit 0
