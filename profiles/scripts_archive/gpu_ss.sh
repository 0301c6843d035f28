#!/bin/bash
# Shared-state hand-off: GPU tests (incl. distributor SIGKILL mid hand-off) + BASELINE config 4 benchmark.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/ss
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_fault_tolerance.py tests/test_gpu_allreduce.py tests/test_shared_state.py -m gpu -v --timeout 200 --timeout-method thread -rf -k "shared_state" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/steps.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u benchmarks/shared_state_sync.py > $OUT/bench_ss.log 2>&1
rc=$?; echo "bench_ss rc=$rc" >> $OUT/steps.log
exit 0
