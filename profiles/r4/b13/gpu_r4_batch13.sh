#!/bin/bash
# Round 4 batch 13: hardware queues per process (GPU_MAX_HW_QUEUES, box default 4) with 8 peers as threads of one
# process. Every peer's copies and kernels share the process's queues, so one peer's last reduce-scatter kernels can
# wait behind the others' queued work (the ~7 ms per-step drain in profiles/r4/b6/qtrace_l1.txt). Separate processes
# per setting (the variable is read at HIP init), alternating, 2 repetitions: quantized ring and plain ring.
# Also: the Python API latency again after async ops initiate on the submitting thread and waits spin first.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b13
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_allreduce.py tests/test_benchmarks.py -m gpu -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u benchmarks/py_latency.py --peers 8 --iters 200 > $OUT/py_latency8.json \
  2> $OUT/py_latency8.err || exit 1
cat $OUT/py_latency8.json
timeout -k 10 200 python -u benchmarks/py_latency.py --peers 2 --iters 200 > $OUT/py_latency2.json \
  2> $OUT/py_latency2.err || exit 1
cat $OUT/py_latency2.json
export PCCL_DISABLE_IPC=1
for rep in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 2 \
      --ops 3 --variants "q$q:" >> $OUT/quant_hwq.jsonl 2> $OUT/quant_hwq${q}_$rep.err || exit 1
    tail -1 $OUT/quant_hwq.jsonl
  done
done
for rep in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u scripts/ring_ab_interleaved.py --pool 2 --windows 2 --ops 5 \
      --variants "q$q:" >> $OUT/ring_hwq.jsonl 2> $OUT/ring_hwq${q}_$rep.err || exit 1
    tail -1 $OUT/ring_hwq.jsonl
  done
done
exit 0
