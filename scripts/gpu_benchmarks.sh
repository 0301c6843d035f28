#!/bin/bash
# BASELINE-config benchmarks on one MI355X (configs 1, 3, 4, 5; config 2 is bench.py). Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" >> gpurun_out/bench_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/bench_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> gpurun_out/bench_steps.log
  tail -n 1 "gpurun_out/bench_$name.log"
  return $rc
}
STEPS=${STEPS:-tests,ss_ipc,ss_tcp,wan,ft,basic}
[[ $STEPS == *tests* ]] && { run tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_benchmarks.py tests/test_gpu_allreduce.py || exit $?; }
[[ $STEPS == *ss_ipc* ]] && { run ss_ipc 300 python benchmarks/shared_state_sync.py --params 1e9 --transport ipc || exit $?; }
[[ $STEPS == *ss_shr* ]] && { run ss_shr 300 python benchmarks/shared_state_sync.py --params 1e9 --transport ipc --shareable || exit $?; }
[[ $STEPS == *ss_tcp* ]] && { run ss_tcp 300 python benchmarks/shared_state_sync.py --params 1e9 --transport tcp || exit $?; }
[[ $STEPS == *wan* ]] && { run wan 400 python benchmarks/wan_quantized.py || exit $?; }
[[ $STEPS == *ft* ]] && { run ft 300 python benchmarks/fault_tolerance.py --log-dir gpurun_out/ft_logs || exit $?; }
[[ $STEPS == *basic* ]] && { run basic 300 python benchmarks/basic_reduce.py || exit $?; }
exit 0
