#!/bin/bash
# Device TCP ring tuning sweep on one GPU (headline config and variants) + rocprofv3 kernel/copy trace of the headline.
# Usage (GPU box): bash profiles/scripts_archive/ring_sweep.sh            (CASES="name|ENV=.. ENV=..|bench args;..." overrides the list)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=$R/gpurun_out/ring
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
CASES=${CASES:-"base|PCCL_TRACE_OPS=1|;p2|PCCL_TRACE_OPS=1|--peers 2;stripes8|PCCL_RING_STRIPES=8|--pool 8;stripes1|PCCL_RING_STRIPES=1|--pool 1;piece16|PCCL_DEVICE_PIECE_BYTES=16777216|"}
IFS=';' read -ra LIST <<< "$CASES"
for c in "${LIST[@]}"; do
  IFS='|' read -r name envs args <<< "$c"
  echo "=== $name env[$envs] args[$args]" >> "$OUT/sweep.log"
  # shellcheck disable=SC2086
  env $envs timeout -k 10 240 python -u bench.py --quick --steps 3 --warmup 1 $args > "$OUT/$name.log" 2>&1
  rc=$?
  grep -h '^{' "$OUT/$name.log" >> "$OUT/sweep.log"
  echo "=== $name rc=$rc" >> "$OUT/sweep.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/prof" -o ring -- \
      python3 "$R/bench.py" --quick --steps 3 --warmup 1 > "$OUT/prof.log" 2>&1
  echo "=== prof rc=$?" >> "$OUT/sweep.log"
fi
exit 0
