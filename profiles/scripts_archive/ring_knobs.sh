#!/bin/bash
# 8-peer device ring: connection pool (stripes) x staging piece size
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/knobs
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for pool in 1 2 4; do
  for piece in 4194304 8388608; do
    PCCL_DEVICE_PIECE_BYTES=$piece timeout -k 10 200 python -u bench.py --quick --steps 5 --warmup 2 --pool $pool > $OUT/p${pool}_${piece}.json 2> $OUT/p${pool}_${piece}.err
    rc=$?; echo "pool=$pool piece=$piece rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/p${pool}_${piece}.json)" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
  done
done
