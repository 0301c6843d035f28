#!/bin/bash
# Round 3: per-step trace marks and a rocprofv3 copy/kernel timeline of the headline device ring.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=gpurun_out/${OUTDIR:-r3_timeline}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
PCCL_TRACE_OPS=1 timeout -k 10 240 python -u bench.py --quick --steps 3 --warmup 1 ${BENCH_ARGS:-} > $OUT/trace.json \
  2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
grep -h "pccl-trace" $OUT/trace.err | tail -8
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d $ROOT/$OUT/prof -o ring -- python3 $ROOT/bench.py --quick --steps 3 --warmup 1 ${BENCH_ARGS:-} \
  > $ROOT/$OUT/prof.log 2>&1 || { tail -20 $ROOT/$OUT/prof.log; exit 1; }
cd $ROOT && python3 scripts/copy_timeline.py $OUT/prof ${BIN_MS:-20} > $OUT/timeline.md && head -12 $OUT/timeline.md
rm -rf $OUT/prof/*/*/*kernel_trace.csv.gz 2>/dev/null; du -sh $OUT/prof
