#!/bin/bash
# Round 5 batch 4: config 3 after spreading single-stripe ops over the whole connection pool (stripe_conn): uint8 at
# 16 / 32 / 64 ops in flight, int8-zps and fp8 at 64 and 128; then config 5 on the xGMI path with every peer's stderr
# kept (the bench's run hit its deadline).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b4}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
wan() { # name cq formats
  log "wan $1"
  timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 --concurrent 8 --stripes 4 \
    --concurrent-quant $2 --repeat 2 --formats $3 > $OUT/wan_$1.json 2> $OUT/wan_$1.err
  rc=$?; log "rc=$rc"; return $rc
}
wan u8_cq16 16 uint8 && wan u8_cq32 32 uint8 && wan u8_cq64 64 uint8 && wan all_cq64 64 int8_zps,fp8 \
  && wan u8_cq128 128 uint8 || exit 1
log "ft ipc"
timeout -k 10 200 python -u benchmarks/fault_tolerance.py --transport ipc --peers 8 --mib 1024 --timeout 140 \
  --log-dir $OUT/ft_ipc_logs > $OUT/ft_ipc.json 2> $OUT/ft_ipc.err
log "rc=$?"
log done
exit 0
