#!/bin/bash
# Small-message path A/B on the GPU box: host ring (2 / 8 peers, 1 KiB) and TCP device ring (8 peers, 64 KiB - 4 MiB)
# with the all-gather path off (PCCL_SMALL_ALLREDUCE_BYTES=0) and on.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/small
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lim in 0 262144; do
  for p in 2 8; do
    PCCL_SMALL_ALLREDUCE_BYTES=$lim timeout -k 10 120 python -u scripts/ipc_latency_trace.py --device cpu --peers $p --kib 1 --iters 300 >> $OUT/host.jsonl 2>> $OUT/err.log || exit $?
    echo "{\"limit\": $lim}" >> $OUT/host.jsonl
  done
done
for lim in 0 67108864; do
  for kib in 64 256 1024 4096; do
    PCCL_DISABLE_IPC=1 PCCL_SMALL_ALLREDUCE_BYTES=$lim timeout -k 10 120 python -u scripts/ipc_latency_trace.py --peers 8 --kib $kib --iters 60 >> $OUT/dev.jsonl 2>> $OUT/err.log || exit $?
    echo "{\"limit\": $lim}" >> $OUT/dev.jsonl
  done
done
exit 0
