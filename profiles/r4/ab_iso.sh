#!/bin/bash
# isolated forward time of libaz variants (AZ_LIB_PATH), alternating:
# bash profiles/r4/ab_iso.sh <rounds> base v1 v2 ...
set -o pipefail
rounds=$1; shift
for r in $(seq $rounds); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/tower_time.py $v || exit 1
  done
done
