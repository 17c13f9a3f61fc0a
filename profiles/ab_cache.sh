#!/bin/bash
# Transposition-cache size A/B on C4 configs[1] (repo root, under gpurun).
set -e
OUT=gpurun_out/ab_cache
mkdir -p $OUT
for c in 25 27; do
  timeout -k 10 300 python3 bench.py --cache-log2 $c --no-cpu-baseline --no-cache-window > $OUT/c4_cache$c.json 2> $OUT/c4_cache$c.err
done
