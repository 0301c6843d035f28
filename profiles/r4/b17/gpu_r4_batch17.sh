#!/bin/bash
# Round 4 batch 17: the driver's N = 2 / 4 / 8 bench launches rehearsed on one MI355X (torchrun ranks on cuda:0,
# PCCL_BENCH_SAME_GPU=1). N = 2 and 4 run their extras in a child per rank, as the driver's run will; N = 8 keeps
# them in the ranks (a child per rank would put 16 processes on the one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b17
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_BENCH_SAME_GPU=1 GPU_MAX_HW_QUEUES=2
for N in 2 4 8; do
  extra=""; [ $N = 8 ] && extra="PCCL_BENCH_EXTRAS_INPROC=1"
  echo "[$(date +%T)] torchrun $N" >> $OUT/steps.log
  env $extra timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29540 + N)) bench.py --gpus $N --steps 10 --warmup 3 --no-peer-curve \
    > $OUT/bench_$N.json 2> $OUT/bench_$N.err
  rc=$?
  echo "[$(date +%T)] N=$N rc=$rc" >> $OUT/steps.log
  [ $rc -eq 0 ] || { tail -30 $OUT/bench_$N.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$N.json')); print($N, d['ms_per_step'], d['value'], sorted(d['extra'].get('multi_gpu_table', {}).keys()))"
done
exit 0
