#!/bin/bash
# Round 3: small-op latency on the xGMI/IPC path without Python in the loop (csrc/tools/latency_native.hip), with
# the library's per-op phase marks (PCCL_TRACE_OPS=1) summarised by scripts/trace_phases.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r3_lat}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
hipcc --offload-arch=gfx950 -O2 -std=c++20 -Iinclude csrc/tools/latency_native.hip -Lpccl_amd/lib -lpccl \
  -Wl,-rpath,$(pwd)/pccl_amd/lib -o /tmp/latency_native || exit 1
port=31000
for cfg in ${CFGS:-"8 1048576" "8 65536" "2 1048576"}; do
  set -- $cfg
  for trace in 0 1; do
    PCCL_TRACE_OPS=$trace timeout -k 10 120 /tmp/latency_native $port $1 $2 ${ITERS:-400} 50 > $OUT/lat_${1}_${2}_t$trace.json \
      2> $OUT/lat_${1}_${2}_t$trace.err || { tail -20 $OUT/lat_${1}_${2}_t$trace.err; exit 1; }
    port=$((port + 100))
    echo "peers=$1 bytes=$2 trace=$trace $(cat $OUT/lat_${1}_${2}_t$trace.json)"
  done
  python3 scripts/trace_phases.py $OUT/lat_${1}_${2}_t1.err 50
done
