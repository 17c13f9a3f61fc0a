#!/bin/bash
# Round-5 GPU session U: (diagnostic) the tower without its weight loads
# (variants/nob.py, wrong outputs) -- how much of the chess one-board tile
# and of the Connect-4 tile the weight stream costs; then chess with one tap
# body (product: compile-time skip word 0) vs three (variants/skwrt.py).
set -o pipefail
out=gpurun_out/r5u
mkdir -p $out
for r in 1 2; do
  for v in base nob; do
    if [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/chess_conv_bench.py 128 20 2>&1 | tail -1 | sed "s/^/$v chess /" | tee -a $out/iso.txt || exit 1
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 456 20 0 2>&1 | tail -1 | sed "s/^/$v c4 /" | tee -a $out/iso.txt || exit 1
  done
done
bash profiles/r5/ab_bench.sh 2 "--game chess" base skwrt 2>&1 | tee $out/ab_chess_skw.txt
