#!/bin/bash
# The whole GPU test suite (as the driver runs it at round end), smoke(), then the driver's bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-suite}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_DEBUG_BACKTRACE_SIGNAL=${PCCL_DEBUG_BACKTRACE_SIGNAL:-1}
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
log pytest
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -rfE \
  > $OUT/pytest_gpu.log 2>&1
rc=$?
log "pytest rc=$rc"
tail -n 15 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
log smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { log "smoke rc=$?"; exit 1; }
if [ "${BENCH:-1}" = 1 ]; then
  log bench
  timeout -k 10 720 python bench.py > $OUT/bench.json 2> $OUT/bench.err
  log "bench rc=$?"
fi
log done
exit $rc
