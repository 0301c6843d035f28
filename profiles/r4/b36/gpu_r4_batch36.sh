#!/bin/bash
# Round 4 batch 36: the GPU fault-tolerance tests incl. the new op_end kills (after the victim's whole part, before
# its completion packet) on the device ring (plain / uint8) and the xGMI path (staged / shareable).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b36
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_fault_tolerance.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -rfE > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; exit $rc
