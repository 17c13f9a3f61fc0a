#!/bin/bash
# chess: kernel trace of a short bench run, per-kernel stats and per-stream chains
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/y
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/y/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --game chess --steps 5 --warmup 5 > gpurun_out/y/bench.json 2> gpurun_out/y/bench.err || exit 1
f=$(find gpurun_out/y/prof -name '*kernel_trace.csv' | head -1); s=$(find gpurun_out/y/prof -name '*kernel_stats.csv' | head -1)
python3 profiles/chain.py $f 0.3 > gpurun_out/y/chain.txt && python3 profiles/busy.py $f 0.3 > gpurun_out/y/busy.txt
cp $s gpurun_out/y/kernel_stats.csv; cat gpurun_out/y/chain.txt; head -20 gpurun_out/y/kernel_stats.csv | cut -c1-200
