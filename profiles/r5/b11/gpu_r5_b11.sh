#!/bin/bash
# Round 5 batch 11: config 3 with the peers' data sockets tuned as remote sockets (kernel buffer autotuning, plain
# sends: what the library does on a real WAN; the relay on 127.0.0.1 made them look same-host) vs the local tuning:
# pools 16 / 32, uint8 at 32 / 64 ops in flight, fp32 at 8.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b11}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pool in ${POOLS:-16 32}; do
  for cq in ${CQS:-32 64}; do
    for tun in remote auto; do
      name=p${pool}_cq${cq}_$tun
      log "$name"
      PCCL_SOCKET_TUNING=$tun timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool $pool \
        --concurrent 8 --stripes 4 --concurrent-quant $cq --repeat 2 --formats fp32,uint8 > $OUT/$name.json 2> $OUT/$name.err
      rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
log done
