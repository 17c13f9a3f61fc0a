#!/bin/bash
# chess forward time of libaz variants (AZ_LIB_PATH), alternating: bash profiles/r4/ab_chess.sh <rounds> base v1 ...
set -o pipefail
rounds=$1; shift
for r in $(seq $rounds); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
    echo -n "$v "; AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/chess_conv_bench.py 128 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
