#!/bin/bash
# Interleaved A/B of one command between an older tree (ab_old/, a git worktree built in-tree: `git worktree add
# ab_old <rev>` + its __graft_entry__.build()) and this tree, on one GPU box: old, new, old, new, ... ($ROUNDS rounds).
#   OUTDIR=<name> ROUNDS=2 LIMIT=300 CMD='python bench.py --quick' bash scripts/gpu_ab.sh
# Outputs gpurun_out/<name>/{old,new}_<i>.json (stdout) and .err; stops at the first failing run.
set -u
R="${GRAFT_REPO_ROOT:-$PWD}"
OUT=$R/gpurun_out/${OUTDIR:-ab}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in $(seq 1 "${ROUNDS:-2}"); do
  for v in old new; do
    if [ $v = old ]; then d=$R/ab_old; else d=$R; fi
    echo "[$(date +%T)] $v $i" >> "$OUT/steps.log"
    (cd "$d" && timeout -k 10 "${LIMIT:-300}" bash -c "$CMD") > "$OUT/${v}_$i.json" 2> "$OUT/${v}_$i.err" || exit $?
  done
done
