#!/bin/bash
# Round 5 batch 19: N = 1 headline (bench.py --quick) with the NUMA binding and PCCL_BENCH_CPU_SPREAD = 2 / 3 / 4 / 8
# CPUs per L3 domain (CCD), interleaved, two passes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b19}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for k in ${KS:-2 3 4 8}; do
    log "pass $pass spread $k"
    PCCL_BENCH_CPU_SPREAD=$k timeout -k 10 300 python bench.py --quick > $OUT/q_p${pass}_k$k.json 2> $OUT/q_p${pass}_k$k.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log done
