#!/bin/bash
# A/B builds of conv16_kernel (macro variants) over M blocks per tile, on the
# self-play / chess / B=4096 shapes.
# Usage (GPU box): bash profiles/micro/conv16_ab.sh <out-dir> "<variant flags>"...
set -o pipefail
out=${1:-gpurun_out/c16ab}
shift
mkdir -p "$out"
for v in "$@"; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 $v profiles/micro/conv16_bench.cpp -o /tmp/c16_$$ || exit 1
  for cfg in "870 6 7" "1000 6 7" "4096 6 7" "256 8 8" "1024 9 9"; do
    for mb in 2 3 4; do
      for mode in 0 1; do
        echo -n "[$v] " >> "$out/ab.txt"
        timeout -k 5 60 /tmp/c16_$$ $cfg $mb $mode 50 >> "$out/ab.txt" || exit 1
      done
    done
  done
done
grep -o '^\[[^]]*\]\|"boards": [0-9]*\|"W": [0-9]\|"wm": [0-9]\|"mode": [0-9]\|"us": [0-9.]*\|"rel": [0-9.e-]*' "$out/ab.txt" | paste -s -d' ' | sed 's/ \[/\n[/g'
