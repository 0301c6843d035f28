#!/bin/bash
# Round 4 batch 24: quantized ring with its reduce-scatter copies on the lane's own stream (default now): GPU tests of
# the quantized paths incl. the kill cases, lanes 1 / 2 / 3 interleaved, and the bench as the driver runs it.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b24
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py tests/test_fault_tolerance.py tests/test_gpu_kernels.py \
  -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "quant or qring or zps or setback" \
  > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
PCCL_DISABLE_IPC=1 timeout -k 10 400 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 4 --ops 3 \
  --variants "l2:PCCL_QUANT_LANES=2;l1:PCCL_QUANT_LANES=1;l3:PCCL_QUANT_LANES=3" > $OUT/lanes.jsonl 2> $OUT/lanes.err || exit 1
cat $OUT/lanes.jsonl
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); e=d['extra']; print(d['ms_per_step'], e['ring_quant_u8_same_peers']['ms_per_op'], e['peer_curve']['DEVICE_RING'])"
exit 0
