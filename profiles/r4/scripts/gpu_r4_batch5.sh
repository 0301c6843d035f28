set -u
QUANT=1 TWO=0 LANES="l1:PCCL_QUANT_LANES=1;l2:PCCL_QUANT_LANES=2;l3:PCCL_QUANT_LANES=3" PIECES="p32:PCCL_QUANT_PIECE_BYTES=33554432" OUTDIR=r4_ab4 bash profiles/r4/scripts/gpu_r4_ab.sh || exit 1
bash profiles/r4/scripts/gpu_r4_latency_ab.sh || exit 1
bash profiles/r4/scripts/gpu_r4_rehearsal.sh || exit 1
