#!/bin/bash
# Round 4 batch 15: quantized ring all-gather consume, kernels reading pinned memory (default) vs copy engine -> HBM
# then de-quantize (as the reduce-scatter does); interleaved in one process, 6 windows. Then the bench (N = 1) with
# the per-process Python latency extra.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b15
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
PCCL_DISABLE_IPC=1 timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 6 --ops 3 \
  --variants "pinned:PCCL_QUANT_AG_STAGED=0;staged:PCCL_QUANT_AG_STAGED=1" > $OUT/ag.jsonl 2> $OUT/ag.err || exit 1
cat $OUT/ag.jsonl
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); e=d['extra']; print(d['ms_per_step'], e['ring_quant_u8_same_peers']['ms_per_op'], e.get('latency_1MiB_ipc_python_processes'))"
exit 0
