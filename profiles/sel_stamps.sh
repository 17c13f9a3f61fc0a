#!/bin/bash
# select_group phase stamps (diagnostic build profiles/ab_libs/selst), network and synthetic evaluators
set -o pipefail
mkdir -p gpurun_out/sel_stamps
export AZ_LIB_PATH=$PWD/profiles/ab_libs/selst/libaz.so
for m in ${MODES:-network synth}; do
  f=""; [ $m = synth ] && f=--synth
  timeout -k 10 300 python3 profiles/sel_stamps.py $f > gpurun_out/sel_stamps/$m.txt 2>&1 || { tail gpurun_out/sel_stamps/$m.txt; exit 1; }
  cat gpurun_out/sel_stamps/$m.txt
done
