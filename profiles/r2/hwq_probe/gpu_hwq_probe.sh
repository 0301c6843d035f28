#!/bin/bash
# 4 processes x 2 peers on one GPU (torchrun rehearsal): does the xGMI/IPC slowdown follow the number of hardware
# queues per process (queue oversubscription across processes)? GPU_MAX_HW_QUEUES 1 / 2 / 4 (box default 4).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/hwq
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_BENCH_SAME_GPU=1
for q in 1 2 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port $((29700 + q)) bench.py --gpus 4 --steps 5 --warmup 2 --no-peer-curve \
    > $OUT/bench_4proc_q$q.out 2> $OUT/bench_4proc_q$q.err
  rc=$?; echo "q=$q rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
