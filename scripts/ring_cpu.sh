#!/bin/bash
# Device TCP ring (headline config, 8 peers x 1 GiB on one GPU): CPU seconds (user / sys) against wall time, to see
# whether the 16-CPU share of the box bounds the loopback TCP ring; spin budget A/B; stripes A/B.
set -u
TIMEFORMAT="real %R user %U sys %S"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ringcpu
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "nproc $(nproc)" > $OUT/env.txt
cat /sys/fs/cgroup/cpu.max >> $OUT/env.txt 2>/dev/null
run() { # name env... -- args
  local name=$1; shift
  echo "=== $name $*" >> $OUT/steps.log
  local t0=$(date +%s.%N)
  { time timeout -k 10 300 env "$@" python -u bench.py --quick --steps 5 --warmup 2 > $OUT/$name.log 2>&1 ; } 2> $OUT/$name.time
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
for v in ${VARIANTS:-base:PCCL_TRACE_OPS=0 poll0:PCCL_EVENT_POLL=0 spin0:PCCL_SPIN_US=0}; do
  run ${v%%:*} ${v#*:}
done
exit 0
