#!/bin/bash
# A/B of the 16-tile kernel's output-channel split (AZ_W16_SPLIT_BELOW: 0 never,
# 512 default = launches under two workgroups per CU, 1000000 always) on the
# forward microbenchmarks, then the forward tests with the split forced.
set -e
for B in 256 700 1000 2000; do for t in 0 512 1000000; do
  echo -n "split_below=$t "; AZ_W16_SPLIT_BELOW=$t timeout -k 10 120 python3 profiles/conv_bench.py $B 30 2>/dev/null | tail -1
done; done
for t in 0 512 1000000; do echo -n "split_below=$t "; AZ_W16_SPLIT_BELOW=$t timeout -k 10 120 python3 profiles/chess_conv_bench.py 256 30 2>/dev/null | tail -1; done
AZ_W16_SPLIT_BELOW=1000000 timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -k "forward or replays" tests/test_chess_selfplay_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
