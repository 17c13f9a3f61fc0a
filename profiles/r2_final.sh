#!/bin/bash
# End-of-round artifacts: GPU suite, default bench (with CPU baselines),
# warmup-60 bench, chess bench.  Usage: bash profiles/r2_final.sh <tag>
set -o pipefail
tag=${1:-r2v}
bash profiles/gpu_check.sh $tag || exit 1
timeout -k 10 300 python bench.py --game chess > gpurun_out/$tag/bench_chess.json 2> gpurun_out/$tag/bench_chess.err || { tail gpurun_out/$tag/bench_chess.err; exit 1; }
tail -c 600 gpurun_out/$tag/bench_chess.json
