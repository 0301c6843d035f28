#!/bin/bash
# One GPU-box session: smoke, GPU tests, 1-GPU bench, rocprofv3 kernel stats. Stops at the first crash / timeout
# (exit codes other than 0 = ok and 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,pytest,bench,prof}
[[ $STEPS == *smoke* ]] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *pytest* ]] && step pytest_gpu 900 python -m pytest tests -m gpu -q -rf --timeout 300
[[ $STEPS == *bench* ]] && step bench 600 python bench.py --steps 10 --warmup 3
if [[ $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  step_dir=$GRAFT_REPO_ROOT/gpurun_out
  echo "=== prof" | tee -a $step_dir/steps.log
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $step_dir/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $step_dir/prof.log 2>&1
  echo "=== prof rc=$?" | tee -a $step_dir/steps.log
fi
exit 0
