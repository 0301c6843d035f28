#!/bin/bash
# Hardware-counter passes (one counter group per run, as the box requires) over the kernel micro-benchmark:
# FETCH_SIZE (HBM bytes read, KB) and WRITE_SIZE (bytes written, KB) per kernel dispatch, with kernel timings.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/pmc"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/$c" -o run -- \
      python3 "$R/scripts/kernel_bench.py" --mib 256 --iters 3 > "$R/gpurun_out/pmc/$c.log" 2>&1 || exit $?
done
