#!/bin/bash
# The other BASELINE.json configs on one MI355X (repo root, under gpurun):
# configs[3] per-GPU shard (C4, 400 sims, 4096 games), configs[3]'s whole
# 32768-game pool on one GPU, configs[2] (Connect-5 9x9, 200 sims, 8192 games).
set -e
OUT=gpurun_out/configs
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --sims 400 --steps 20 --warmup 40 --no-cpu-baseline --no-cache-window > $OUT/s400.json 2> $OUT/s400.err
timeout -k 10 600 python3 bench.py --sims 400 --slots 32768 --cache-log2 27 --steps 10 --warmup 30 --no-cpu-baseline --no-cache-window > $OUT/s400_32k.json 2> $OUT/s400_32k.err
timeout -k 10 600 python3 bench.py --height 9 --width 9 --n 5 --sims 200 --slots 8192 --steps 10 --warmup 30 --no-cpu-baseline --no-cache-window > $OUT/c5_9x9.json 2> $OUT/c5_9x9.err
