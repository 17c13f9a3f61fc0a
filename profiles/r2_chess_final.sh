#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2i/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2i/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2i/gpu_tests.log
timeout -k 10 300 python bench.py --game chess > gpurun_out/r2i/bench_chess.json 2> gpurun_out/r2i/bench_chess.err || { tail gpurun_out/r2i/bench_chess.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r2i/bench_chess.json').read().strip().splitlines()[-1]); print('chess', d['value'], d['roofline']['frac'], d.get('gpu_over_cpu'))"
