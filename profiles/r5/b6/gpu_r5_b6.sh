#!/bin/bash
# Round 5 batch 6: the driver's bench on the reordered tree (multi-process measurements before the bench's own GPU
# context; extra.per_rank), config 5 on the xGMI path with PCCL_TRACE_OPS (the 111 ms ops between rejoin and
# re-solve), and the N = 8 launch rehearsed on one GPU (8 torchrun ranks, one peer each, extra.per_rank).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b6}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
if [ "${BENCH:-1}" = 1 ]; then
  log bench
  timeout -k 10 720 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { log "bench rc=$?"; exit 1; }
fi
log "ft ipc trace"
PCCL_TRACE_OPS=1 timeout -k 10 200 python -u benchmarks/fault_tolerance.py --transport ipc --peers 8 --mib 1024 \
  --timeout 140 --log-dir $OUT/ft_ipc_logs > $OUT/ft_ipc.json 2> $OUT/ft_ipc.err
log "rc=$?"
if [ "${REHEARSAL:-1}" = 1 ]; then
  log "rehearsal 8"
  PCCL_BENCH_SAME_GPU=1 GPU_MAX_HW_QUEUES=2 PCCL_BENCH_EXTRAS_INPROC=1 timeout -k 10 900 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 10 \
    --warmup 3 --no-peer-curve > $OUT/rehearsal_8.json 2> $OUT/rehearsal_8.err
  log "rc=$?"
fi
log done
exit 0
