#!/bin/bash
# Rehearsal of the driver's multi-GPU bench path on one GPU: torchrun with 2 and 4 processes (PCCL_BENCH_SAME_GPU=1:
# every rank on cuda:0), full extras (xGMI/IPC between processes with shareable buffers, sweeps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/torchrun
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_BENCH_SAME_GPU=1
for n in ${NPROCS:-2 4}; do
  timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 > $OUT/bench_${n}proc.out 2> $OUT/bench_${n}proc.err
  rc=$?; echo "n=$n rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
