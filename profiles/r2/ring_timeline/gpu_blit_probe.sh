#!/bin/bash
# Which copies of the headline ring run as ROCclr blit kernels? rocprofv3 kernel + memory-copy trace of a short run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=gpurun_out/blit
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d $ROOT/$OUT/prof -o ring -- python3 $ROOT/bench.py --quick --steps 2 --warmup 1 > $ROOT/$OUT/prof.log 2>&1
echo "rc=$?" >> $ROOT/$OUT/steps.log
