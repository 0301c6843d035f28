#!/bin/bash
# Round 4: interleaved in-process A/B runs (scripts/ring_ab_interleaved.py) of the quantized device ring's lane count
# and piece size at 8 peers x 1 GiB, a per-step trace of the quantized ring (PCCL_TRACE_OPS), and the 2-peer plain
# device ring over piece sizes / pool sizes with its per-step trace.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r4_ab}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
AB="python -u scripts/ring_ab_interleaved.py"
run() { # name timeout args...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.jsonl 2> $OUT/$name.err
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.log
  cat $OUT/$name.jsonl
  return $rc
}
if [ "${QUANT:-1}" = 1 ]; then
  run quant_lanes 300 $AB --quant --windows 4 --ops 3 \
    --variants "${LANES:-l1:PCCL_QUANT_LANES=1;l2:PCCL_QUANT_LANES=2;l3:PCCL_QUANT_LANES=3;l4:PCCL_QUANT_LANES=4}" || exit 1
  run quant_piece 300 $AB --quant --windows 4 --ops 3 \
    --variants "${PIECES:-p4:PCCL_QUANT_PIECE_BYTES=4194304;p8:PCCL_QUANT_PIECE_BYTES=8388608;p16:PCCL_QUANT_PIECE_BYTES=16777216}" || exit 1
  PCCL_TRACE_OPS=1 run quant_trace 200 $AB --quant --windows 1 --ops 2 --warmup 1 --variants "base:" || exit 1
fi
if [ "${TWO:-1}" = 1 ]; then
  for pool in ${POOLS:-4 8}; do
    run two_pool$pool 300 $AB --peers 2 --pool $pool --windows 4 --ops 5 \
      --variants "${TWO_PIECES:-p16:PCCL_DEVICE_PIECE_BYTES=16777216;p32:PCCL_DEVICE_PIECE_BYTES=33554432;p64:PCCL_DEVICE_PIECE_BYTES=67108864}" || exit 1
  done
  PCCL_TRACE_OPS=1 run two_trace 200 $AB --peers 2 --pool 8 --windows 1 --ops 3 --warmup 1 --variants "base:" || exit 1
fi
exit 0
