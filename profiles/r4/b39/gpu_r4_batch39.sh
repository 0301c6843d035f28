#!/bin/bash
# Round 4 batch 39: the bench's per-process Python latency with the peer processes on 2 hardware queues each (the
# slow mode, ~545 us, showed up inside the bench, where the bench process itself also holds the GPU's queues).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b39
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); e=d['extra']; print(d['ms_per_step'], e['ring_quant_u8_same_peers']['ms_per_op'], e['latency_1MiB_ipc_python_processes'], e['latency_1MiB_ipc_us'])"
exit 0
