#!/bin/bash
# Round 5 batch 7: config 3 with aligned per-op connection groups (stripe_conn + op_stripes): uint8 at 16 / 32 / 64 /
# 128 ops in flight, then every format at the chosen concurrency, and fp32 at 8 ops.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b7}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
wan() { # name cq formats [extra args]
  local name=$1 cq=$2 fm=$3; shift 3
  log "wan $name"
  timeout -k 10 300 python -u benchmarks/wan_quantized.py --mib 2048 --pool 16 --concurrent 8 --stripes 4 \
    --concurrent-quant $cq --repeat 2 --formats $fm "$@" > $OUT/wan_$name.json 2> $OUT/wan_$name.err
  rc=$?; log "rc=$rc"; return $rc
}
wan u8_cq16 16 uint8 && wan u8_cq32 32 uint8 && wan u8_cq64 64 uint8 && wan u8_cq128 128 uint8 \
  && wan all_cq${CQ:-64} ${CQ:-64} fp32,uint8,int8_zps,fp8 || exit 1
log done
