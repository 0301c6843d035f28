#!/bin/bash
# Bench with progress + periodic thread stacks (PCCL_BENCH_WATCHDOG): shareable buffers on / off.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/bdiag
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_BENCH_WATCHDOG=40
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > $OUT/bench_shr.out 2> $OUT/bench_shr.err
echo "shr rc=$?" >> $OUT/steps.log
PCCL_SHAREABLE_BUFFERS=0 timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > $OUT/bench_noshr.out 2> $OUT/bench_noshr.err
echo "noshr rc=$?" >> $OUT/steps.log
exit 0
