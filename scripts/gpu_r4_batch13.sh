#!/bin/bash
# Round 4 batch 13: hardware queues per process (GPU_MAX_HW_QUEUES, box default 4) with 8 peers as threads of one
# process. Every peer's copies and kernels share the process's queues, so one peer's last reduce-scatter kernels can
# wait behind the others' queued work (the ~7 ms per-step drain in profiles/r4/b6/qtrace_l1.txt). Separate processes
# per setting (the variable is read at HIP init), alternating, 2 repetitions: quantized ring and plain ring.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4_b13
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DISABLE_IPC=1
for rep in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 2 \
      --ops 3 --variants "q$q:" >> $OUT/quant_hwq.jsonl 2> $OUT/quant_hwq${q}_$rep.err || exit 1
    tail -1 $OUT/quant_hwq.jsonl
  done
done
for rep in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u scripts/ring_ab_interleaved.py --pool 2 --windows 2 --ops 5 \
      --variants "q$q:" >> $OUT/ring_hwq.jsonl 2> $OUT/ring_hwq${q}_$rep.err || exit 1
    tail -1 $OUT/ring_hwq.jsonl
  done
done
exit 0
