#!/bin/bash
# GPU box: IPC tests (safe VMM default + fast), fault tests with kill + rejoin, fault-tolerance benchmark on IPC.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/b3
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name" >> $OUT/steps.log; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_ipc 500 python -u -m pytest tests/test_gpu_allreduce.py tests/test_fault_tolerance.py -m gpu -x -v --timeout 200 --timeout-method thread
run fault_bench_ipc 300 python -u benchmarks/fault_tolerance.py --peers 8 --mib 64 --log-dir $OUT/ft_logs
exit 0
