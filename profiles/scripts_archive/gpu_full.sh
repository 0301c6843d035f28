#!/bin/bash
# GPU box: full GPU test suite, 1-GPU bench (headline + extras child), torchrun rehearsal of the multi-GPU bench path
# on one GPU (2 processes, PCCL_BENCH_SAME_GPU=1). Stops at the first crash / timeout (pytest rc 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/full
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" >> $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
[[ ${STEPS:-pytest,bench,torchrun} == *pytest* ]] && step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -rf
[[ ${STEPS:-pytest,bench,torchrun} == *bench* ]] && step bench 600 python -u bench.py --steps ${BENCH_STEPS:-10} --warmup 3
[[ ${STEPS:-pytest,bench,torchrun} == *torchrun* ]] && PCCL_BENCH_SAME_GPU=1 step torchrun2 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --mib 256
exit 0
