#!/bin/bash
# 1-GPU bench with the ring pool pinned to 2 (round-2 default for 8 peers) vs per-phase auto sizing, then the torchrun
# rehearsal (2 / 4 processes on one GPU). Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/pool
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --pool 2 > $OUT/bench_pool2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench_auto.log 2>&1 || exit $?
bash scripts/gpu_torchrun.sh
