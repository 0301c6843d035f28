#!/bin/bash
# Round 4: device-ring pipeline (pruned to one strategy) and quantized ring v2 (lanes, cut-through all-gather) on one
# MI355X: ring GPU tests, mid-op SIGKILL tests of the device ring, the GPU ring stress run, then the headline bench
# and the quantized ring at 8 peers x 1 GiB.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r4_ring}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.log
  tail -n 4 $OUT/$name.log
  return $rc
}
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
# a test failure (rc 1) goes on to the next step; a timeout, crash or fault (any other rc) ends the call
ok() { [ $1 -le 1 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step ring_tests 900 $PYT tests/test_gpu_allreduce.py -m gpu -k "${K:-ring or quantized or two_peers or concurrent}"; ok $? || exit 1
  step quant_kernels 400 $PYT tests/test_gpu_kernels.py -m gpu -k "quant"; ok $? || exit 1
  step quarantine 300 $PYT tests/test_fault_tolerance.py -m gpu -k "quarantine"; ok $? || exit 1
  step ring_kills 900 $PYT tests/test_fault_tolerance.py -m gpu -k "ring_sigkill"; ok $? || exit 1
  step ring_stress 300 $PYT tests/test_stress.py -m gpu -k "gpu_ring"; ok $? || exit 1
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench_ring 400 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-ipc-extra --no-peer-curve || exit 1
  cp $OUT/bench_ring.log $OUT/bench_ring.json 2>/dev/null
fi
exit 0
