#!/bin/bash
# conv16_kernel phase clocks per tile (diagnostic stamp build; GPU box)
set -o pipefail
out=gpurun_out/c16phase.txt; mkdir -p gpurun_out; : > $out
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DAZ_C16_STAMPS profiles/micro/conv16_bench.cpp -o /tmp/c16s || exit 1
for cfg in "887 6 7 3 0" "887 6 7 3 1" "887 6 7 2 0" "887 6 7 4 0" "256 8 8 2 0" "4096 6 7 4 0"; do
  echo "[$cfg]" >> $out
  timeout -k 5 60 /tmp/c16s $cfg 30 >> $out 2>&1 || exit 1
done
grep -o '^\[.*\]\|stamps.*\|"us": [0-9.]*' $out
