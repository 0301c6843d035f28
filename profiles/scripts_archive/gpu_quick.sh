#!/bin/bash
# Short GPU check: selected GPU tests (-k filter in $K) then the device-ring sweep (profiles/scripts_archive/ring_sweep.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/${TESTS:-test_gpu_allreduce.py} -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_quick.log 2>&1
rc=$?
tail -n 5 gpurun_out/pytest_quick.log
[ $rc -ne 0 ] && exit $rc
[ "${SWEEP:-1}" = 1 ] && bash profiles/scripts_archive/ring_sweep.sh
exit 0
