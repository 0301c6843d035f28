#!/bin/bash
# rocprofv3 evidence for the flagship bench on one GPU, into gpurun_out/${OUTDIR:-prof}/:
#   trace/  kernel + memory-copy trace stats of the headline (bench.py --quick: TCP device ring, 8 peers x 1 GiB bf16)
#   qtrace/ kernel stats of the uint8-quantized device ring (scripts/ring_ab_interleaved.py)
#   pmc_*/  one PMC pass per counter group (FETCH_SIZE takes 3 of the 4 TCC counters, WRITE_SIZE 2): HBM bytes
# Summaries: python scripts/prof_summary.py / scripts/pmc_summary.py on the CSVs.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=$R/gpurun_out/${OUTDIR:-prof}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
log() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
cd /tmp && export TMPDIR=/tmp
log trace
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace" -o ring -- \
  python3 "$R/bench.py" --quick --steps 5 --warmup 2 > "$OUT/trace.log" 2>&1 || { log "trace rc=$?"; exit 1; }
log "quant trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/qtrace" -o quant -- \
  python3 "$R/scripts/ring_ab_interleaved.py" --quant --variants "u8:" --windows 2 --ops 3 --warmup 2 \
  > "$OUT/qtrace.log" 2>&1 || log "qtrace rc=$?"
for c in FETCH_SIZE WRITE_SIZE; do
  log "pmc $c"
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o ring -- \
    python3 "$R/bench.py" --quick --steps 3 --warmup 1 > "$OUT/pmc_$c.log" 2>&1 || { log "pmc $c rc=$?"; break; }
done
log done
