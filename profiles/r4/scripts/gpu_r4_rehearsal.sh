#!/bin/bash
# Round 4: rehearsal of the N > 1 bench path on one MI355X: 8 torchrun ranks on cuda:0 (PCCL_BENCH_SAME_GPU=1), one
# peer per rank, headline + extras incl. extra.multi_gpu_table (RCCL skipped: the ranks share one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r4_rehearsal}
mkdir -p $OUT
# extras in the ranks themselves: a child per rank would put 16 processes on the one GPU
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_BENCH_SAME_GPU=1 GPU_MAX_HW_QUEUES=2 PCCL_BENCH_EXTRAS_INPROC=1
N=${NPROC:-8}
echo "[$(date +%T)] torchrun $N" >> $OUT/steps.log
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port ${PORT:-29533} bench.py --gpus $N --steps ${STEPS:-10} --warmup 3 --no-peer-curve \
  > $OUT/bench_$N.json 2> $OUT/bench_$N.err
rc=$?
echo "[$(date +%T)] rc=$rc" >> $OUT/steps.log
tail -c 3000 $OUT/bench_$N.json
exit $rc
