#!/bin/bash
# A/B on one box: device-ring staging piece size (PCCL_DEVICE_PIECE_BYTES) for the headline (8 peers x 1 GiB, 2 stripes).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/piece_ab
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in ${REPS:-1 2}; do
  for mib in ${PIECES:-8 16 32 4}; do
    PCCL_DEVICE_PIECE_BYTES=$((mib << 20)) timeout -k 10 240 python -u bench.py --quick --steps 10 --warmup 3 \
      > $OUT/piece${mib}_run$i.log 2>&1 || exit $?
    echo "piece=${mib}MiB run=$i $(grep -h 'done:' $OUT/piece${mib}_run$i.log | tail -1)" >> $OUT/summary.txt
  done
done
