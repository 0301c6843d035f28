#!/bin/bash
# Sweep of the xGMI push-kernel knobs for threaded peers sharing one GPU (scripts/ipc_knob_sweep.py per setting).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ipc_knobs
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { # label env...
  local label=$1; shift
  env "$@" timeout -k 10 180 python -u scripts/ipc_knob_sweep.py >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || { echo "$label failed" >> $OUT/steps.log; exit 1; }
  echo "$label ok" >> $OUT/steps.log
}
run default PCCL_IPC_DUMMY=0
run default2 PCCL_IPC_DUMMY=1
run grid64 PCCL_IPC_GRID=64
run grid128 PCCL_IPC_GRID=128
run grid512 PCCL_IPC_GRID=512
run unroll4 PCCL_IPC_UNROLL=4
run tiled4 PCCL_IPC_TILED=1 PCCL_IPC_UNROLL=4
run tiled2 PCCL_IPC_TILED=1 PCCL_IPC_UNROLL=2
exit 0
