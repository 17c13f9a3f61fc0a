#!/bin/bash
# A/B the conv3x3_mfma variants (AZ_CONV_VARIANT, csrc/az_nn.hip launch_forward),
# two interleaved rounds, forward microbenchmark at B=4096.
set -e
for round in 1 2; do
  for v in ${VARIANTS:-0 1 2 5 6}; do
    echo -n "variant $v round $round: "
    AZ_CONV_VARIANT=$v timeout -k 10 120 python3 profiles/conv_bench.py 4096 20 2>/dev/null | tail -1
  done
done
