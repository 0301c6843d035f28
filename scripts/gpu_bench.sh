#!/bin/bash
# The driver's bench exactly as it runs it (python bench.py, defaults), plus smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-bench}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "[$(date +%T)] smoke" >> $OUT/steps.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
echo "[$(date +%T)] bench" >> $OUT/steps.log
timeout -k 10 720 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "[$(date +%T)] rc=$rc" >> $OUT/steps.log
exit $rc
