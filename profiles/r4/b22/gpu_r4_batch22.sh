#!/bin/bash
# Round 4 batch 22: per-step trace of the quantized ring (lanes 2, current kernels), for the per-step latency
# breakdown (q = payload quantized and published, f = first piece of the step consumed, rs / ag = step done).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b22
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
PCCL_TRACE_OPS=1 timeout -k 10 300 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 1 --ops 3 \
  --warmup 2 --variants "base:" > $OUT/qtrace.jsonl 2> $OUT/qtrace.err || exit 1
grep -c "pccl-trace" $OUT/qtrace.err
exit 0
