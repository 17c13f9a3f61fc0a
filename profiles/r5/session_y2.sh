#!/bin/bash
# chess: kernel trace of the current build (per-stream chains), then policy dense NB=1 vs 2
set -o pipefail
mkdir -p gpurun_out/y2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/y2/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --game chess --steps 5 --warmup 5 > gpurun_out/y2/bench.json 2> gpurun_out/y2/bench.err || exit 1
f=$(find gpurun_out/y2/prof -name '*kernel_trace.csv' | head -1)
python3 profiles/chain.py $f 0.3 > gpurun_out/y2/chain.txt && cat gpurun_out/y2/chain.txt
find gpurun_out/y2/prof -name '*kernel_trace.csv' -delete
bash profiles/r5/ab_bench.sh 2 "--game chess" base pd1 2>&1 | tee gpurun_out/y2/ab_pd1.txt
