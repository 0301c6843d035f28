#!/bin/bash
# Round 5 batch 23: CPU mask of the bench's one-process-per-peer TCP runs (full / spread / numa), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b23}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "[$(date +%T)] masks" >> $OUT/steps.log
timeout -k 10 1000 python -u profiles/r5/b23/r5_config_masks.py > $OUT/masks.jsonl 2> $OUT/masks.err
echo "[$(date +%T)] rc=$?" >> $OUT/steps.log
