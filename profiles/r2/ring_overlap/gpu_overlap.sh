#!/bin/bash
# rocprofv3 timeline of the headline device ring (kernels, copies, roctx op ranges + per-frame send/recv ranges) and
# its overlap summary (scripts/ring_overlap.py).
set -u
ROOT="${GRAFT_REPO_ROOT:-$PWD}"
OUT=$ROOT/gpurun_out/overlap
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PCCL_ROCTX_IO=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d $OUT/prof -o ring \
  -- python3 $ROOT/bench.py --quick --steps 2 --warmup 1 > $OUT/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
ls -R $OUT/prof > $OUT/files.txt
P=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 $ROOT/scripts/ring_overlap.py ${P%_kernel_trace.csv} > $OUT/overlap.md 2>&1
echo "analysis rc=$?" >> $OUT/steps.log
exit 0
