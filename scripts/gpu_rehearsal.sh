#!/bin/bash
# The driver's N > 1 launch rehearsed on one GPU (PCCL_BENCH_SAME_GPU=1): torchrun with N ranks, the extras
# in a child process per rank (as on a real node), extra.per_rank and extra.multi_gpu_table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-rehearsal}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_BENCH_SAME_GPU=1 GPU_MAX_HW_QUEUES=2
N=${NPROC:-2}
echo "[$(date +%T)] torchrun $N" >> $OUT/steps.log
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port ${PORT:-29533} bench.py --gpus $N --steps ${STEPS:-10} --warmup 3 > $OUT/bench_$N.json 2> $OUT/bench_$N.err
rc=$?
echo "[$(date +%T)] rc=$rc" >> $OUT/steps.log
tail -c 2000 $OUT/bench_$N.json
exit $rc
