#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/peer_ccd
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3; do
  for v in 0 1; do
    PCCL_BENCH_PEER_CCD=$v timeout -k 10 200 python bench.py --quick --steps 10 --warmup 3 --windows 2 > $OUT/v${v}_r$rep.json 2> $OUT/v${v}_r$rep.err || { tail -20 $OUT/v${v}_r$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('$OUT/v${v}_r$rep.json').read().strip().splitlines()[-1]);e=d['extra'];print('ccd=$v rep=$rep', d['ms_per_step'], e['windows_ms'], e['cpu_cores_busy_rank0'])"
  done
done
