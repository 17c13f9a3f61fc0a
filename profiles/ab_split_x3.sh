#!/bin/bash
# The bf16x3 kernel with hardware bf16 conversion (v_cvt_pk_bf16_f32 split):
# forward parity tests, then the output-channel split threshold
# (AZ_W16_SPLIT_BELOW) on the microbenchmarks and end to end.
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -k "forward or replays" tests/test_chess_selfplay_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
timeout -k 10 120 python3 profiles/net_error.py 2>&1 | tail -3
for B in 700 1000 2000 4096; do for t in 640 1000000; do
  echo -n "split_below=$t "; AZ_W16_SPLIT_BELOW=$t timeout -k 10 120 python3 profiles/conv_bench.py $B 30 2>/dev/null | tail -1
done; done
for t in 640 1000 1600; do
  echo -n "split_below=$t C4 bench: "; AZ_W16_SPLIT_BELOW=$t timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['unit'], d['roofline']['achieved'])"
done
for t in 640 1000000; do
  echo -n "split_below=$t chess bench: "; AZ_W16_SPLIT_BELOW=$t timeout -k 10 300 python3 bench.py --game chess --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['unit'])"
done
