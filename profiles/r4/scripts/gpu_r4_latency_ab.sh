#!/bin/bash
# Round 4: small-op latency of the xGMI path (pccl_latency, C API, threaded peers on cuda:0) at 64 KiB and 1 MiB,
# interleaved 4 times (the round-3 table had 64 KiB slower than 1 MiB from separate runs).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r4_latency}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3 4; do
  for b in 65536 1048576 16777216; do
    for p in 8 2; do
      port=$((31000 + rep * 100 + p))
      timeout -k 10 60 pccl_amd/lib/pccl_latency $port $p $b 300 50 >> $OUT/lat.jsonl 2>> $OUT/lat.err || exit 1
    done
  done
done
cat $OUT/lat.jsonl
