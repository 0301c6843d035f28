#!/bin/bash
# Round 4: BASELINE config 3 through the WAN emulator: relay calibration with plain streams (no library), then the
# library's quantized / fp32 all-reduce through the relay at several in-flight settings (8 peers on cuda:0).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r4_wan}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "[$(date +%T)] calibrate" >> $OUT/steps.log
[ "${CALIBRATE:-1}" = 1 ] && { timeout -k 10 200 python -u scripts/wan_relay_calibrate.py --conns ${CONNS:-16,32,64,128} --seconds 6 > $OUT/calibrate.jsonl 2> $OUT/calibrate.err || exit 1; cat $OUT/calibrate.jsonl; }
for cfg in ${CFGS:-16:8:4:32 16:8:4:16 16:8:4:64}; do
  IFS=: read pool conc stripes cq <<< "$cfg"
  name=p${pool}_c${conc}_s${stripes}_cq${cq}
  echo "[$(date +%T)] $name" >> $OUT/steps.log
  timeout -k 10 400 python -u benchmarks/wan_quantized.py --mib ${MIB:-2048} --pool $pool --concurrent $conc \
    --stripes $stripes --concurrent-quant $cq --formats ${FORMATS:-fp32,uint8,int8_zps,fp8} > $OUT/$name.json 2> $OUT/$name.err
  rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.log
  tail -c 1500 $OUT/$name.json
  [ $rc -eq 0 ] || exit $rc
done
exit 0
