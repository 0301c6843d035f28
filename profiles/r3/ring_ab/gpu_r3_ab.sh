#!/bin/bash
# Round 3: interleaved A/B of headline-ring knobs (8 peers x 1 GiB). Each variant: "<label>|<env assignments>|<bench args>"
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r3_ab}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
IFS=';' read -ra VS <<< "${VARIANTS:-base||}"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    IFS='|' read -r label envs args <<< "$v"
    env $envs timeout -k 10 ${AB_TIMEOUT:-240} python -u bench.py ${QUICK---quick} --steps ${STEPS:-10} --warmup 3 $args > $OUT/$label.$rep.json \
      2> $OUT/$label.$rep.err || { tail -20 $OUT/$label.$rep.err; exit 1; }
    echo "$label rep=$rep $(python3 -c "import json;d=json.load(open('$OUT/$label.$rep.json'));e=d['extra'];print(d['ms_per_step'], 'ms', e['cpu_cores_busy_rank0'], 'cores', {k: v['ms'] for k, v in e.get('sweep', {}).get('DEVICE_RING', {}).items()})")"
  done
done
