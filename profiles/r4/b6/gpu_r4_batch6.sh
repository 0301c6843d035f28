#!/bin/bash
# Round 4 batch 6: quantized ring per-step trace (fine marks), quantized ring at 2 vs 4 connections per neighbour,
# and the WAN benchmark with CPU peers (host ring) pipelined vs step-synchronous (PCCL_TMP_STEPWISE, temporary A/B).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b6
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB="python -u scripts/ring_ab_interleaved.py"
PCCL_DISABLE_IPC=1 PCCL_TRACE_OPS=1 PCCL_QUANT_LANES=1 timeout -k 10 200 $AB --quant --windows 1 --ops 2 --warmup 1 \
  --variants "base:" > $OUT/qtrace_l1.jsonl 2> $OUT/qtrace_l1.err || exit 1
PCCL_DISABLE_IPC=1 PCCL_TRACE_OPS=1 timeout -k 10 200 $AB --quant --windows 1 --ops 2 --warmup 1 \
  --variants "base:" > $OUT/qtrace_l2.jsonl 2> $OUT/qtrace_l2.err || exit 1
for pool in 2 4 8; do
  PCCL_DISABLE_IPC=1 timeout -k 10 200 $AB --quant --pool $pool --windows 3 --ops 3 --variants "pool$pool:" \
    > $OUT/qpool$pool.jsonl 2> $OUT/qpool$pool.err || exit 1
  cat $OUT/qpool$pool.jsonl
done
for rep in 1 2; do
  for m in pipe step; do
    if [ $m = step ]; then export PCCL_TMP_STEPWISE=1; else unset PCCL_TMP_STEPWISE; fi
    timeout -k 10 300 python -u benchmarks/wan_quantized.py --device cpu --mib 1024 --formats fp32 \
      > $OUT/wan_cpu_${m}_$rep.json 2> $OUT/wan_cpu_${m}_$rep.err || exit 1
    tail -c 600 $OUT/wan_cpu_${m}_$rep.json
  done
done
unset PCCL_TMP_STEPWISE
exit 0
