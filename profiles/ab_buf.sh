#!/bin/bash
# wino16x with buffer loads (chunk offsets in soffset, range-checked zero
# padding): full GPU suite, network error, forward microbenchmarks, benches.
set -e
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_buf_tests.log 2>&1
tail -2 gpurun_out/ab_buf_tests.log
timeout -k 10 120 python3 profiles/net_error.py 2>&1 | tail -2
for B in 700 1000 2000 4096; do
  timeout -k 10 120 python3 profiles/conv_bench.py $B 30 2>/dev/null | tail -1
done
timeout -k 10 120 python3 profiles/chess_conv_bench.py 256 30 2>/dev/null | tail -1
for i in 1 2; do
  echo -n "C4 bench: "; timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['unit'], d['roofline']['achieved'])"
  echo -n "chess bench: "; timeout -k 10 300 python3 bench.py --game chess --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['unit'])"
done
