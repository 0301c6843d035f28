#!/bin/bash
# Round 3: device-ring pipeline check on one MI355X — ring GPU tests, then headline A/B (send-ahead pipeline,
# step-0 staging queue) and the 2-peer point over connection pool sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-r3_ring}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_allreduce.py -x -v --timeout 150 --timeout-method thread \
    -k "${TESTS:-ring or two_peers or concurrent}" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
for v in ${VARIANTS:-1:1 0:1 1:0}; do
  a=${v%%:*}; s=${v##*:}
  PCCL_RING_SEND_AHEAD=$a PCCL_RING_STEP0_OP_STREAM=$s timeout -k 10 240 python -u bench.py --quick --steps 10 \
    --warmup 3 > $OUT/bench_a${a}_s${s}.json 2> $OUT/bench_a${a}_s${s}.err || { tail -20 $OUT/bench_a${a}_s${s}.err; exit 1; }
  echo "8 peers ahead=$a step0_op_stream=$s $(grep -h 'done:' $OUT/bench_a${a}_s${s}.err | tail -1)"
done
for pool in ${POOLS2:-2 4 8}; do
  timeout -k 10 120 python -u bench.py --quick --peers 2 --pool $pool --steps 10 --warmup 3 > $OUT/bench2_p$pool.json \
    2> $OUT/bench2_p$pool.err || { tail -20 $OUT/bench2_p$pool.err; exit 1; }
  echo "2 peers pool=$pool $(grep -h 'done:' $OUT/bench2_p$pool.err | tail -1)"
done
