#!/bin/bash
# GPU/IPC elastic soak: reference schedule (every 0.5-2 s spawn p=0.6 / SIGKILL p=0.4, >= 2 alive) for SOAK_S seconds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/soak
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_STRESS_SECONDS=${SOAK_S:-600}
timeout -k 10 $((PCCL_STRESS_SECONDS + 240)) python -u -m pytest tests/test_stress.py -m gpu -s -v --timeout $((PCCL_STRESS_SECONDS + 200)) --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "rc=$?" >> $OUT/steps.log
