#!/bin/bash
# Round 5 batch 2: smoke + the driver's bench on HEAD, then BASELINE config 3 (uint8 through the WAN relay) at 16 / 32 /
# 64 ops in flight, each multi-op run twice (cold pools, then warm) with staging-pool allocation counters.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b2}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
if [ "${BENCH:-1}" = 1 ]; then
  log smoke
  timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { log "smoke rc=$?"; exit 1; }
  log bench
  timeout -k 10 720 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { log "bench rc=$?"; exit 1; }
fi
for cq in ${CQS:-16 32 64}; do
  log "wan cq=$cq"
  timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib ${MIB:-2048} --pool 16 --concurrent 8 --stripes 4 \
    --concurrent-quant $cq --repeat 2 --formats ${FORMATS:-uint8} > $OUT/wan_cq$cq.json 2> $OUT/wan_cq$cq.err
  rc=$?
  log "wan cq=$cq rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
log done
exit 0
