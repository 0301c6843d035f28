#!/bin/bash
# Round 5 batch 32: blocking stream-ordered calls with the xGMI kernels on the caller's stream
# (PCCL_CALLER_STREAM_KERNELS=1) vs a pooled library stream, 8 peer processes, 1 MiB, interleaved over two passes;
# then the stream-ordered GPU tests with the knob on.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r5b32}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> $OUT/steps.log; }
for pass in 1 2; do
  for v in pooled caller; do
    log "pass $pass $v"
    if [ $v = caller ]; then export PCCL_CALLER_STREAM_KERNELS=1; else unset PCCL_CALLER_STREAM_KERNELS; fi
    timeout -k 10 240 python -u benchmarks/py_latency.py --peers 8 --iters 300 --sizes 1048576 \
      > $OUT/lat_p${pass}_$v.json 2> $OUT/lat_p${pass}_$v.err
    rc=$?; log "rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
export PCCL_CALLER_STREAM_KERNELS=1
log pytest
timeout -k 10 400 python -u -m pytest tests/test_gpu_allreduce.py tests/test_ddp_overlap.py -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "stream or ddp or ipc or producer or in_place or inplace" > $OUT/pytest.log 2>&1
rc=$?; log "pytest rc=$rc"
