#!/bin/bash
# GPU box: xGMI/IPC GPU tests, then SIGKILL a peer at fixed protocol points (inside the push kernel, right after its
# vote) for out-of-place and in-place 1 GiB bf16 ops across 3 processes; each probe prints a JSON summary.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ipc_fault
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ipc_fault/pytest.log 2>&1
  rc=$?; tail -n 3 gpurun_out/ipc_fault/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
CASES=${CASES:-oop_kernel:ipc_kernel:300: inp_kernel:ipc_kernel:300:--inplace oop_vote:ipc_vote:300: inp_vote:ipc_vote:300:--inplace}
for c in $CASES; do
  IFS=: read -r name point seq extra <<< "$c"
  timeout -k 10 100 python -u scripts/ipc_kill_probe.py --inject "$point:$seq" --duration 6 $extra \
      --out gpurun_out/ipc_fault/$name > gpurun_out/ipc_fault/$name.json 2> gpurun_out/ipc_fault/$name.err
  rc=$?
  echo "$name rc=$rc $(cat gpurun_out/ipc_fault/$name.json)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
