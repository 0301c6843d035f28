#!/bin/bash
# A/B on one box: ring receive loop parked on one stripe (PCCL_RING_GROUP_WAIT=0) vs woken by any stripe (1).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/groupwake_ab
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  for gw in 0 1; do
    for p in 8 2; do
      PCCL_RING_GROUP_WAIT=$gw timeout -k 10 240 python -u bench.py --quick --steps 10 --warmup 3 --peers $p \
        > $OUT/gw${gw}_p${p}_run$i.log 2>&1 || exit $?
      echo "gw=$gw peers=$p run=$i $(grep -h 'done:' $OUT/gw${gw}_p${p}_run$i.log | tail -1)" >> $OUT/summary.txt
    done
  done
done
