#!/bin/bash
# shared-state hand-off tests (packed staging, kills) + torchrun rehearsal of the multi-GPU bench (2 / 4 procs)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/b5
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_fault_tolerance.py tests/test_gpu_allreduce.py -m gpu -v --timeout 200 --timeout-method thread -rf -k "shared_state or small_messages" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/steps.log; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_torchrun.sh
