#!/bin/bash
# Round 5 batch 18: the N = 1 headline with the bench bound to the GPU's NUMA node (PCCL_BENCH_NUMA_BIND=1, on top
# of the per-CCD CPU spread) vs unbound, alternating, two passes each (bench.py --quick: headline only).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b18}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for nb in 0 1; do
    log "pass $pass numa $nb"
    PCCL_BENCH_NUMA_BIND=$nb timeout -k 10 300 python bench.py --quick > $OUT/q_p${pass}_n$nb.json 2> $OUT/q_p${pass}_n$nb.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log done
