#!/bin/bash
# shareable-memory tests + bench (progress + watchdog) + ring CPU accounting
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/b4
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -v --timeout 120 --timeout-method thread -rf -k "shareable or threaded" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/steps.log; [ $rc -le 1 ] || exit $rc
PCCL_BENCH_WATCHDOG=60 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $OUT/bench.out 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ring_cpu.sh
