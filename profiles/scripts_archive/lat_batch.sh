#!/bin/bash
# Control-path latency after master send coalescing + timer slack: IPC (safe/fast) and host ring, 2 and 8 peers.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/lat2
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash profiles/scripts_archive/tcp_loopback.sh || exit $?
for p in 2 8; do
  timeout -k 10 120 python -u scripts/ipc_latency_trace.py --device cpu --peers $p --kib 1 --iters 300 >> $OUT/lat.jsonl 2>> $OUT/lat.err || exit $?
  for mode in safe fast; do
    PCCL_IPC_MODE=$mode timeout -k 10 120 python -u scripts/ipc_latency_trace.py --peers $p --kib 64 --iters 300 >> $OUT/lat.jsonl 2>> $OUT/lat.err || exit $?
  done
done
exit 0
