#!/bin/bash
# Ring receive loop waiting on all stripes at once: bench twice + the ring / IPC GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/groupwake
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench_1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench_2.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py tests/test_hierarchical.py tests/test_fault_tolerance.py -m gpu -v --timeout 170 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/steps.log
