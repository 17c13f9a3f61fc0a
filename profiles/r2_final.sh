#!/bin/bash
# End-of-round artifacts: GPU suite, default bench (with CPU baselines), warmup-60 bench, chess bench.
set -o pipefail
bash profiles/gpu_check.sh r2j || exit 1
timeout -k 10 300 python bench.py --game chess > gpurun_out/r2j/bench_chess.json 2> gpurun_out/r2j/bench_chess.err || { tail gpurun_out/r2j/bench_chess.err; exit 1; }
tail -c 600 gpurun_out/r2j/bench_chess.json
