#!/bin/bash
# Round 4 batch 12: the late-abort restore (OpState::settle) on the GPU paths (ring / qring kills incl. the 3:end
# cases, IPC kills, in-place device tests), the Python API's per-op latency with one process per peer, and the
# quantized ring's lane count with the fused quantize + owner-parity kernel.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b12
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_fault_tolerance.py tests/test_gpu_allreduce.py -m gpu -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider -k "sigkill or kill or inplace or in_place or restore" \
  > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u benchmarks/py_latency.py --peers 8 --iters 200 > $OUT/py_latency8.json \
  2> $OUT/py_latency8.err || exit 1
cat $OUT/py_latency8.json
timeout -k 10 200 python -u benchmarks/py_latency.py --peers 2 --iters 200 > $OUT/py_latency2.json \
  2> $OUT/py_latency2.err || exit 1
cat $OUT/py_latency2.json
PCCL_DISABLE_IPC=1 timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 4 --ops 3 \
  --variants "l1:PCCL_QUANT_LANES=1;l2:PCCL_QUANT_LANES=2;l3:PCCL_QUANT_LANES=3;l4:PCCL_QUANT_LANES=4" \
  > $OUT/quant_lanes.jsonl 2> $OUT/quant_lanes.err || exit 1
cat $OUT/quant_lanes.jsonl
exit 0
