#!/bin/bash
# Round 4: rocprofv3 kernel + copy timeline of the quantized device ring (8 peers x 1 GiB, uint8) and of the 2-peer
# plain device ring, summarised per time bin by scripts/copy_timeline.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=gpurun_out/${OUTDIR:-r4_prof}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
prof() { # name args...
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
    --output-format csv -d $ROOT/$OUT/$name -o run -- python3 $ROOT/scripts/ring_ab_interleaved.py "$@" \
    > $ROOT/$OUT/$name.log 2>&1) || { tail -20 $OUT/$name.log; return 1; }
  python3 scripts/copy_timeline.py $OUT/$name ${BIN_MS:-10} > $OUT/$name.timeline.md
  head -40 $OUT/$name.timeline.md
  rm -f $OUT/$name/*/*/*kernel_trace.csv $OUT/$name/*/*/*memory_copy_trace.csv 2>/dev/null
  return 0
}
prof quant8 --quant --windows 1 --ops 2 --warmup 1 --variants "${QV:-p16:PCCL_QUANT_PIECE_BYTES=16777216}" || exit 1
prof two2 --peers 2 --pool 8 --windows 1 --ops 3 --warmup 1 --variants "base:" || exit 1
exit 0
