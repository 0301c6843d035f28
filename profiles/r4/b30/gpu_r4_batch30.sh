#!/bin/bash
# Round 4 batch 30: quantized ring copies chosen by step size (lane stream for >= 4 MiB quantized steps, else the
# shared queue / pinned reads): GPU quantized tests, the bench-size ring, and config 3 over the WAN emulator.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r4_b30
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py tests/test_fault_tolerance.py tests/test_benchmarks.py \
  -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "quant or qring or wan" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
PCCL_DISABLE_IPC=1 timeout -k 10 300 python -u scripts/ring_ab_interleaved.py --quant --pool 2 --windows 4 --ops 3 \
  --variants "base:" > $OUT/ring.jsonl 2> $OUT/ring.err || exit 1
cat $OUT/ring.jsonl
CALIBRATE=0 OUTDIR=r4_b30/wan CFGS="16:8:4:32 16:8:4:16" bash profiles/r4/scripts/gpu_r4_wan.sh > $OUT/wan.log 2>&1 || exit 1
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4_b30/wan/*.json")):
    d = json.load(open(f))
    print(f, {k: round(v["seconds"], 3) for k, v in d["formats"].items()})
PY
exit 0
