#!/bin/bash
# A/B of the bf16x3-term Winograd kernel (AZ_WINO_X3=1, az_wino16x.hip) vs the
# fp32-MFMA 16-tile kernel: forward tests with it forced, microbenchmarks,
# end-to-end benches.
set -e
AZ_WINO_X3=1 timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -k "forward or replays" tests/test_chess_selfplay_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
for B in 256 700 1000 2000 4096; do for x in 0 1; do
  echo -n "x3=$x "; AZ_WINO_X3=$x timeout -k 10 120 python3 profiles/conv_bench.py $B 30 2>/dev/null | tail -1
done; done
for x in 0 1; do echo -n "x3=$x "; AZ_WINO_X3=$x timeout -k 10 120 python3 profiles/chess_conv_bench.py 256 30 2>/dev/null | tail -1; done
for x in 0 1; do
  echo -n "x3=$x C4 bench: "; AZ_WINO_X3=$x timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['unit'])"
  echo -n "x3=$x chess bench: "; AZ_WINO_X3=$x timeout -k 10 300 python3 bench.py --game chess --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['unit'])"
done
