#!/bin/bash
# Phase latency of small IPC all-reduces (scripts/ipc_latency_trace.py): safe and fast IPC modes, 2 and 8 peers.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/lat
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for mode in safe fast; do
  for p in 2 8; do
    for kib in 64 1024; do
      PCCL_IPC_MODE=$mode timeout -k 10 120 python -u scripts/ipc_latency_trace.py --peers $p --kib $kib --iters 200 >> $OUT/lat.jsonl 2>> $OUT/lat.err || exit $?
    done
  done
done
timeout -k 10 300 python -u bench.py --peers 2 --quick --steps 10 --warmup 3 > $OUT/bench_ring_2peers.log 2>&1 || exit $?
exit 0
