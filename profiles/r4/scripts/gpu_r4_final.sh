#!/bin/bash
# Round 4 checkpoint: bench.py exactly as the driver runs it (N = 1), then the whole GPU test suite and smoke().
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r4_final}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "[$(date +%T)] bench" >> $OUT/steps.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "[$(date +%T)] bench rc=$rc" >> $OUT/steps.log
tail -c 400 $OUT/bench.json
[ $rc -eq 0 ] || exit $rc
OUTDIR=${OUTDIR:-r4_final} bash profiles/r4/scripts/gpu_r4_fulltests.sh
