#!/bin/bash
# Profiles the flagship bench on one GPU: per-op phase trace (PCCL_TRACE_OPS) + rocprofv3 kernel stats.
# Usage (on the GPU box): bash scripts/gpu_prof.sh [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PCCL_TRACE_OPS=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --rejoin 0 "$@" > gpurun_out/trace.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --rejoin 0 "$@" > "$R/gpurun_out/prof.log" 2>&1
# roctx ranges (one per collective / shared-state sync) and phase markers next to the kernels
[ "${MARKERS:-1}" = 1 ] && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
    -d "$R/gpurun_out/prof_markers" -o bench -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --rejoin 0 "$@" > "$R/gpurun_out/prof_markers.log" 2>&1
