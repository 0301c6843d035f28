#!/bin/bash
# Loopback-TCP cost on the GPU box: throughput and CPU seconds per GB vs socket buffer size, hot vs cold buffers;
# then the headline ring with per-thread CPU accounting.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r3_tcp}
mkdir -p $OUT
g++ -O2 -std=c++20 -pthread csrc/tools/tcp_loopback_probe.cpp -o /tmp/tcpl || exit 1
{ echo "nproc $(nproc) quota $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; for f in core/rmem_max core/wmem_max ipv4/tcp_rmem ipv4/tcp_wmem core/optmem_max; do echo "$f $(cat /proc/sys/net/$f 2>/dev/null)"; done; uname -r; } > $OUT/env.txt
IFS=';' read -ra PL <<< "${PROBES:-8 2 0 1;8 2 0 0;8 1 0 1;8 2 2048 1;2 4 0 1;2 8 0 1;2 8 0 0}"
for v in "${PL[@]}"; do
  [ -z "$v" ] && continue
  set -- $v
  timeout -k 5 120 ${PREFIX:-} /tmp/tcpl $1 $2 1024 4096 $3 $4 >> $OUT/tcpl.jsonl 2>&1 || exit $?
done
cat $OUT/tcpl.jsonl
if [ "${BENCH:-1}" = 1 ]; then
  export HSA_ENABLE_IPC_MODE_LEGACY=0
  cat /sys/fs/cgroup/cpu.stat > $OUT/cpu_stat_before.txt 2>&1
  timeout -k 10 240 ${PREFIX:-} python -u bench.py --quick --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat /sys/fs/cgroup/cpu.stat > $OUT/cpu_stat_after.txt 2>&1
  paste $OUT/cpu_stat_before.txt $OUT/cpu_stat_after.txt
  python3 -c "import json;d=json.load(open('$OUT/bench.json'));e=d['extra'];print(d['ms_per_step'],e['cpu_cores_busy_rank0']);print(json.dumps(e['cpu_by_thread_rank0']))"
fi
