#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/nanogpt
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u benchmarks/nanogpt_ddp.py --iters 30 > $OUT/ddp.json 2> $OUT/ddp.err; echo "ddp rc=$?" >> $OUT/steps.log
timeout -k 10 400 python -u benchmarks/nanogpt_ddp.py --iters 30 --overlap > $OUT/ddp_overlap.json 2> $OUT/ddp_overlap.err; echo "overlap rc=$?" >> $OUT/steps.log
timeout -k 10 300 python -u benchmarks/nanogpt_ddp.py --iters 30 --peers 1 > $OUT/single.json 2> $OUT/single.err; echo "single rc=$?" >> $OUT/steps.log
exit 0
