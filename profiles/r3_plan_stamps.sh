#!/bin/bash
# phase stamps with and without the slot plan (per-wave K-loop spans)
set -o pipefail
mkdir -p gpurun_out/r3_plan_stamps
for p in 0 1; do
  echo "== AZ_TOWER_PLAN=$p"
  AZ_TOWER_PLAN=$p AZ_LIB_PATH=$PWD/profiles/ab_libs/stamps/libaz.so timeout -k 10 120 python profiles/tower_stamps.py 4096 2>&1 | grep -v amdgpu.ids | grep -E "B=|wave [0-7]" || exit 1
done | tee gpurun_out/r3_plan_stamps/stamps.txt
