#!/bin/bash
# Round 5 batch 25: where the stream-ordered small ops lose against `ready`: py_latency with per-op traces, then the
# same without traces (the tracing's own cost), 8 peer processes over the xGMI path, 1 MiB bf16.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b25}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
log traced
timeout -k 10 240 python -u benchmarks/py_latency.py --peers 8 --iters 300 --sizes 1048576 --trace-dir $OUT/traces \
  > $OUT/py_latency_traced.json 2> $OUT/py_latency_traced.err
rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 0 3 7; do python profiles/r5/b25/lat_variant_phases.py $OUT/traces/peer$r.err all_reduce,async,ready > $OUT/phases_peer$r.jsonl; done
log plain
timeout -k 10 240 python -u benchmarks/py_latency.py --peers 8 --iters 300 --sizes 1048576 \
  > $OUT/py_latency_plain.json 2> $OUT/py_latency_plain.err
rc=$?; log "rc=$rc"
