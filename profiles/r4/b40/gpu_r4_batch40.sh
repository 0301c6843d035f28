#!/bin/bash
# Round 4 batch 40: GPU benchmark-script tests on HEAD (py_latency peers on 2 hardware queues each) and smoke().
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b40
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_benchmarks.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -rfE > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 200 python -u benchmarks/py_latency.py --peers 8 --iters 200 --sizes 1048576 > $OUT/py_latency8.json 2>&1 || exit 1
cat $OUT/py_latency8.json
exit 0
