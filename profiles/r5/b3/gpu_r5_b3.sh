#!/bin/bash
# Round 5 batch 3: BASELINE config 3 (uint8, 50 ms WAN relay) at 16 / 32 / 64 ops in flight with slab staging pools,
# small reduce-scatter steps staged through the shared copy queue (copy) vs de-quantized from pinned memory (pinned);
# then the collocated-sites emulation (5 ms one way, 50 Gbit/s links, 10 Gbit/s flows): relay calibration and fp32 at
# 4 and 8 peers.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b3}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for mode in ${MODES:-copy pinned}; do
  for cq in ${CQS:-16 32 64}; do
    log "wan $mode cq=$cq"
    PCCL_QUANT_SMALL_RS=$mode timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 \
      --concurrent 8 --stripes 4 --concurrent-quant $cq --repeat 2 --formats ${FORMATS:-uint8} \
      > $OUT/wan_${mode}_cq$cq.json 2> $OUT/wan_${mode}_cq$cq.err
    rc=$?
    log "rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
if [ "${COLO:-1}" = 1 ]; then
  log calibrate_colo
  timeout -k 10 200 python -u scripts/wan_relay_calibrate.py --delay-ms 5 --flow-mbit 10000 --link-mbit 50000 \
    --conns 8,16,32 --seconds 5 > $OUT/calibrate_colo.jsonl 2> $OUT/calibrate_colo.err || { log "calibrate rc=$?"; exit 1; }
  for peers in 4 8; do
    log "colo fp32 peers=$peers"
    timeout -k 10 300 python -u benchmarks/wan_quantized.py --peers $peers --mib 2048 --latency-ms 5 \
      --flow-mbit 10000 --link-mbit 50000 --pool 16 --concurrent 8 --repeat 2 --formats fp32,uint8 \
      > $OUT/colo_p$peers.json 2> $OUT/colo_p$peers.err
    rc=$?
    log "rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
log done
exit 0
