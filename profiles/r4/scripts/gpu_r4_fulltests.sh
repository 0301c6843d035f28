#!/bin/bash
# Round 4: the whole GPU test suite (as the driver runs it at round end) plus smoke(), one pytest process.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r4_fulltests}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -rfE \
  > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -n 15 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc2=$?
tail -n 3 $OUT/smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
