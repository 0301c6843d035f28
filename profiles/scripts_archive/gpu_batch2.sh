#!/bin/bash
# GPU box: stress (IPC) + fault tests, fault-tolerance benchmark (BASELINE config 5) on the IPC path, kernel bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/b2
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name" >> $OUT/steps.log; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_stress_fault 400 python -u -m pytest tests/test_stress.py tests/test_fault_tolerance.py -m gpu -v --timeout 200 --timeout-method thread
run fault_bench_ipc 300 python -u benchmarks/fault_tolerance.py --peers 8 --mib 64 --log-dir $OUT/ft_logs
run kbench 200 python -u scripts/kernel_bench.py
exit 0
