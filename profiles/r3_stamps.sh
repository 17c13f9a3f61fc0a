#!/bin/bash
# tower phase clocks (AZ_T16_STAMPS build) with the slot plan, B = 673 and 4096
set -o pipefail
mkdir -p gpurun_out/r3_stamps
for nb in 673 4096; do
  AZ_LIB_PATH=$PWD/profiles/ab_libs/stamps/libaz.so timeout -k 10 120 python profiles/tower_stamps.py $nb 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r3_stamps/stamps.txt || exit 1
done
