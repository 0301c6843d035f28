#!/bin/bash
# Round 3: interleaved in-process A/B of device-ring knobs (scripts/ring_ab_interleaved.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-r3_abi}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PCCL_DISABLE_IPC=1
n=0
IFS='#' read -ra SETS <<< "${SETS:-l1:PCCL_RING_LANES=1;l2:PCCL_RING_LANES=2;l3:PCCL_RING_LANES=3}"
for set in "${SETS[@]}"; do
  n=$((n + 1))
  timeout -k 10 ${ABI_TIMEOUT:-300} python -u scripts/ring_ab_interleaved.py --variants "$set" --windows ${WINDOWS:-6} \
    --ops ${OPS:-4} ${ABI_ARGS:-} > $OUT/set$n.jsonl 2> $OUT/set$n.err || { tail -20 $OUT/set$n.err; exit 1; }
  cat $OUT/set$n.jsonl
done
