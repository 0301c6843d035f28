#!/bin/bash
# Round 5 batch 26: the 8-process small-op latency with 1 vs 2 hardware queues per process (GPU_MAX_HW_QUEUES),
# interleaved; then one traced run with 1 queue.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b26}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for q in 1 2; do
    log "pass $pass hwq $q"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u benchmarks/py_latency.py --peers 8 --iters 300 --sizes 1048576 \
      > $OUT/lat_p${pass}_q$q.json 2> $OUT/lat_p${pass}_q$q.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
log traced
GPU_MAX_HW_QUEUES=1 timeout -k 10 240 python -u benchmarks/py_latency.py --peers 8 --iters 300 --sizes 1048576 \
  --trace-dir $OUT/traces > $OUT/lat_traced_q1.json 2> $OUT/lat_traced_q1.err
rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 0 3 7; do python profiles/r5/b25/lat_variant_phases.py $OUT/traces/peer$r.err all_reduce,async,ready > $OUT/phases_q1_peer$r.jsonl; done
log done
