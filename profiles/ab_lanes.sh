#!/bin/bash
# Lane-count A/B on the end-of-round build (repo root, under gpurun):
# C4 configs[1] with 2 (auto) vs 3 lanes, chess configs[4] shard with 1 (auto) vs 2.
set -e
OUT=gpurun_out/ab_lanes
mkdir -p $OUT
for l in 2 3; do
  timeout -k 10 300 python3 bench.py --lanes $l --steps 20 --warmup 40 --no-cpu-baseline --no-cache-window > $OUT/c4_l$l.json 2> $OUT/c4_l$l.err
done
for l in 1 2; do
  timeout -k 10 300 python3 bench.py --game chess --lanes $l --no-cpu-baseline > $OUT/chess_l$l.json 2> $OUT/chess_l$l.err
done
