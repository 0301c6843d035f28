#!/bin/bash
# Kernel throughput table at the current tree + rocprofv3 kernel stats of the same bench (device-side durations).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=gpurun_out/kernels
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/kernel_bench.py --mib 512 --iters 20 > $OUT/kernels.md 2> $OUT/kernels.err || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/$OUT/prof -o kb -- python3 $ROOT/scripts/kernel_bench.py --mib 512 --iters 5 > $ROOT/$OUT/prof.log 2>&1
echo "prof rc=$?" >> $ROOT/$OUT/steps.log
