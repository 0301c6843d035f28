#!/bin/bash
# Round 3: interleaved A/B of an env knob on the xGMI/IPC small-op latency (pccl_latency, no Python in the loop).
# VARIANTS="name:ENV=V,ENV2=V2;name2:..." ; CFGS="8 1048576" ; REPS=3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-r3_lat_ab}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=32000
IFS=';' read -ra VS <<< "${VARIANTS:-spin0:PCCL_MASTER_RX_SPIN_US=0;spin200:PCCL_MASTER_RX_SPIN_US=200}"
for rep in $(seq 1 ${REPS:-3}); do
  for cfg in ${CFGS:-"8 1048576" "2 1048576"}; do
    set -- $cfg
    for v in "${VS[@]}"; do
      name=${v%%:*}; envs=${v#*:}
      env $(echo $envs | tr ',' ' ') timeout -k 10 120 pccl_amd/lib/pccl_latency $port $1 $2 ${ITERS:-400} 50 \
        > $OUT/${name}_${1}_${2}_r$rep.json 2> $OUT/${name}_${1}_${2}_r$rep.err || { tail -20 $OUT/${name}_${1}_${2}_r$rep.err; exit 1; }
      port=$((port + 50))
      echo "$name peers=$1 bytes=$2 rep=$rep $(cat $OUT/${name}_${1}_${2}_r$rep.json)"
    done
  done
done
