#!/bin/bash
# Round 4 batch 20: 32-bit conversions in the quantize / de-quantize helpers (no 64-bit FP64 emulation for wire types
# up to 32 bits; ZPS in 32-bit integers up to 16-bit types): device vs host bit-exactness for every type, the kernel
# table, and the quantized ring.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=gpurun_out/r4_b20
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_allreduce.py -m gpu -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "quant or zps or setback" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/$OUT/prof -o kb -- python3 $ROOT/scripts/kernel_bench.py --mib 512 --iters 5 > $ROOT/$OUT/prof.log 2>&1) || exit 1
rm -f $OUT/prof/kb_kernel_trace.csv
PCCL_DISABLE_IPC=1 timeout -k 10 300 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 4 --ops 3 \
  --variants "base:" > $OUT/quant.jsonl 2> $OUT/quant.err || exit 1
cat $OUT/quant.jsonl
exit 0
