#!/bin/bash
# Loopback TCP ceiling on the GPU box (csrc/tools/tcp_loopback_probe.cpp): ring of P peers, C connections per link.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/tcpl
mkdir -p $OUT
g++ -O2 -std=c++20 -pthread csrc/tools/tcp_loopback_probe.cpp -o /tmp/tcpl || exit 1
echo "nproc $(nproc) affinity $(python -c 'import os; print(len(os.sched_getaffinity(0)))')" > $OUT/env.txt
for p in 2 8; do
  for c in 1 2 4 8; do
    timeout -k 5 120 /tmp/tcpl $p $c 1024 >> $OUT/tcpl.jsonl 2>&1 || exit $?
  done
done
exit 0
