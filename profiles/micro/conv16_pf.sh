#!/bin/bash
# conv16_kernel weight-prefetch depth (AZ_C16_PF) over tile heights, chess and C4 launch sizes (GPU box)
set -o pipefail
out=gpurun_out/c16pf.txt; mkdir -p gpurun_out; : > $out
for pf in 2 3 4 6 8; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DAZ_C16_PF=$pf profiles/micro/conv16_bench.cpp -o /tmp/c16pf || exit 1
  for cfg in "256 8 8 2 1" "256 8 8 2 0" "887 6 7 3 1" "887 6 7 3 0" "4096 6 7 4 1"; do
    echo -n "[PF=$pf] " >> $out
    timeout -k 5 60 /tmp/c16pf $cfg 50 >> $out || exit 1
  done
done
grep -o '^\[[^]]*\]\|"boards": [0-9]*\|"wm": [0-9]\|"mode": [0-9]\|"us": [0-9.]*\|"rel": [0-9.e-]*' $out | paste -s -d' ' | sed 's/ \[/\n[/g'
