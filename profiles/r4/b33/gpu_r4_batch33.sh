#!/bin/bash
# Round 4 batch 33: what separates the fast (~125-190 us) and slow (~550 us) runs of the 8-process Python latency:
# 6 repetitions with the cgroup's throttling counters per run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b33
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u profiles/scripts_archive/lat_mode_probe.py --reps 6 > $OUT/modes.jsonl 2> $OUT/modes.err || exit 1
cat $OUT/modes.jsonl
exit 0
