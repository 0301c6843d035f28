#!/bin/bash
# Round 3 checkpoint: GPU test suite (driver's command) + full bench (driver's command), outputs under gpurun_out/<OUTDIR>.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r3_full}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print("value", d["value"], d["unit"], "ms/op", d["ms_per_step"], "windows", e.get("windows_ms"), "cores", e.get("cpu_cores_busy_rank0"))
print("curve", json.dumps(e.get("peer_curve")))
print("ipc", json.dumps(e.get("ipc_same_peers")), "lat1MiB", e.get("latency_1MiB_ipc_us"), "cfg1", e.get("latency_cpu_4elem_2peers"))
PY
