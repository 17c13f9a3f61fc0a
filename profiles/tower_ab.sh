#!/bin/bash
# build A/B variants of libaz: bash profiles/tower_ab.sh build name "-DFLAG=.." ...; run: bash profiles/tower_ab.sh run name...
set -o pipefail
cmd=$1; shift
if [ "$cmd" = build ]; then
  while [ $# -gt 0 ]; do
    v=$1; flags=$2; shift 2
    make -s -j8 -C custom-alphazero_amd/csrc OBJDIR=_obj_$v OUT=../../profiles/ab_libs/$v/libaz.so EXTRA="$flags" || exit 1
  done
else
  mkdir -p gpurun_out/tower_ab
  for v in "$@"; do
    if [ "$v" = base ]; then lib=custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=profiles/ab_libs/$v/libaz.so; fi
    AZ_LIB_PATH=$PWD/$lib timeout -k 10 120 python profiles/tower_time.py $v || exit 1
  done
fi
