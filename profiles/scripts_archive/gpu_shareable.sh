#!/bin/bash
# Shareable (VMM + fd) buffers on the xGMI path: memory-module / threaded / two-process tests, SIGKILL-mid-kernel with
# shareable buffers, then the 1-GPU bench with extras. Stops at the first crash / timeout (pytest rc 1 = failures).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/shr
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" >> $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_shr 600 python -u -m pytest tests/test_gpu_allreduce.py tests/test_fault_tolerance.py -m gpu -v --timeout 200 --timeout-method thread -rf -k "shareable or threaded or two_process_ipc or sigkill"
step bench 600 python -u bench.py --steps ${BENCH_STEPS:-5} --warmup 2
exit 0
