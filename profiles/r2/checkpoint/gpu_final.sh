#!/bin/bash
# Round checkpoint on one MI355X: smoke, full GPU test suite, 1-GPU bench (headline + extras), rocprofv3 kernel +
# copy stats of the headline ring, BASELINE-config benchmarks. Stops at a crash / timeout (rc 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=gpurun_out/final
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
S=${STEPS:-smoke,pytest,bench,prof,benchmarks}
[[ $S == *smoke* ]] && step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
[[ $S == *pytest* ]] && step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -rf
[[ $S == *bench* ]] && step bench 600 python -u bench.py --steps 10 --warmup 3
if [[ $S == *prof* ]]; then
  (cd /tmp && export TMPDIR=/tmp && step_name=prof && \
   timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $ROOT/$OUT/prof -o ring \
     -- python3 $ROOT/bench.py --quick --steps 3 --warmup 1 > $ROOT/$OUT/prof.log 2>&1; echo "=== prof rc=$?" >> $ROOT/$OUT/steps.log)
fi
[[ $S == *benchmarks* ]] && STEPS=ss_ipc,ss_shr,ss_tcp,ft,basic step benchmarks 1200 bash scripts/gpu_benchmarks.sh
exit 0
