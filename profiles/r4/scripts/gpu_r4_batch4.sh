set -u
QUANT=1 TWO=0 LANES="l1:PCCL_QUANT_LANES=1;l2:PCCL_QUANT_LANES=2" PIECES="p16:PCCL_QUANT_PIECE_BYTES=16777216;p32:PCCL_QUANT_PIECE_BYTES=33554432;p64:PCCL_QUANT_PIECE_BYTES=67108864" OUTDIR=r4_ab3 bash profiles/r4/scripts/gpu_r4_ab.sh || exit 1
CALIBRATE=0 OUTDIR=r4_wan2 bash profiles/r4/scripts/gpu_r4_wan.sh || exit 1
bash profiles/r4/scripts/gpu_r4_rehearsal.sh || exit 1
