#!/bin/bash
# Round 3: BASELINE config 3 (8 peers, 2 GiB fp32 each, 50 ms one-way WAN, 25 Gbit/s link, 1 Gbit/s per flow) with
# the WAN emulated by a separate relay process (pccl_wan_relay) and, for comparison, by the in-library model.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUTDIR:-r3_wan}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for emu in ${EMUS:-relay builtin}; do
  timeout -k 10 ${WAN_TIMEOUT:-400} python -u benchmarks/wan_quantized.py --emulator $emu ${WAN_ARGS:-} > $OUT/wan_$emu.json 2> $OUT/wan_$emu.err \
    || { tail -20 $OUT/wan_$emu.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/wan_$emu.json').read().strip().splitlines()[-1]);print('$emu', d['wan'].get('relayed_GB'), {k:(v['seconds'],v['ref_metric_rx_plus_tx_Gbit_per_peer']) for k,v in d['formats'].items()})"
done
