#!/bin/bash
# Device-ring send-ahead: GPU tests of the device ring paths, then bench A/B (ahead on / off) at 8 and 2 peers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ahead
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
PCCL_RING_SEND_AHEAD=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_allreduce.py tests/test_hierarchical.py tests/test_wan.py -m gpu -v --timeout 200 --timeout-method thread -rf -k "ring or concurrent or disable_ipc or two_peers or hierarchical or quantized or three_peers" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest (send-ahead) rc=$rc" >> $OUT/steps.log; [ $rc -le 1 ] || exit $rc
for a in 1 0; do
  for p in 8 2; do
    PCCL_RING_SEND_AHEAD=$a timeout -k 10 200 python -u bench.py --peers $p --quick --steps 5 --warmup 2 > $OUT/ring_${p}p_ahead$a.json 2> $OUT/ring_${p}p_ahead$a.err
    rc=$?; echo "ahead=$a peers=$p rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
