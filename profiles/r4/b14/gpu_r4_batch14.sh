#!/bin/bash
# Round 4 batch 14: A/B of the async-op change (initiate on the submitting thread, spinning waits) on one box:
# ab_old/libpccl.so = the commit before it (same build flags), the in-tree library = after; the same HIP plugin.
# Python API latency, one process per peer, 8 and 2 peers, alternating, 3 repetitions.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b14
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_HIP_PLUGIN=$PWD/pccl_amd/lib/libpccl_hip.so
for rep in 1 2 3; do
  for v in old new; do
    lib=$PWD/pccl_amd/lib/libpccl.so; [ $v = old ] && lib=$PWD/ab_old/libpccl.so
    for p in 8 2; do
      PCCL_LIBRARY=$lib timeout -k 10 200 python -u benchmarks/py_latency.py --peers $p --iters 200 \
        --sizes 65536,1048576 > $OUT/lat_${v}_${p}_$rep.json 2> $OUT/lat_${v}_${p}_$rep.err || exit 1
      python3 -c "import json; d=json.load(open('$OUT/lat_${v}_${p}_$rep.json')); print('$v', $p, {k: (r['all_reduce']['median_us'], r['ready']['median_us']) for k, r in d['sizes'].items()})"
    done
  done
done
exit 0
