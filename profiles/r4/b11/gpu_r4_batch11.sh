#!/bin/bash
# Round 4 batch 11: fused quantize + owner parity kernel tests, the quantized ring with it (A/B is against the previous
# checkpoint's 207 ms), and the 2-peer device ring with the per-CCD CPU spread vs the full CPU mask (separate
# processes, alternating).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b11
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_allreduce.py -m gpu -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "setback or quant" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
PCCL_DISABLE_IPC=1 timeout -k 10 300 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 4 --ops 3 \
  --variants "base:" > $OUT/quant.jsonl 2> $OUT/quant.err || exit 1
cat $OUT/quant.jsonl
for rep in 1 2 3; do
  for sp in 3 0; do
    PCCL_BENCH_CPU_SPREAD=$sp timeout -k 10 200 python -u bench.py --peers 2 --quick --steps 10 --warmup 3 \
      > $OUT/two_sp${sp}_$rep.json 2> $OUT/two_sp${sp}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$OUT/two_sp${sp}_$rep.json')); print('spread $sp', d['ms_per_step'], d['extra']['windows_ms'])"
  done
done
exit 0
