#!/bin/bash
# diagnostic: the older waves (0-3) take the second M half (AZ_T16_SWAPMH):
# does the K-loop lead follow the wave's age or the M half's content?
set -o pipefail
mkdir -p gpurun_out/r3_swapmh
AZ_LIB_PATH=$PWD/profiles/ab_libs/st_swap/libaz.so timeout -k 10 120 python profiles/tower_stamps.py 4096 2>&1 | grep -v amdgpu.ids | grep -E "B=|wave [0-7]" | tee gpurun_out/r3_swapmh/stamps.txt
