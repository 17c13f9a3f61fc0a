#!/bin/bash
# A/B the residual-tower conv variants (AZ_CONV_VARIANT, csrc/az_nn.hip
# launch_forward: 0 Winograd, 6 direct default, 1-5 direct tilings / DIAG),
# two interleaved rounds, forward microbenchmark at each batch size in $BATCHES.
set -e
for B in ${BATCHES:-4096}; do
  for round in 1 2; do
    for v in ${VARIANTS:-0 6}; do
      echo -n "variant $v round $round: "
      AZ_CONV_VARIANT=$v timeout -k 10 120 python3 profiles/conv_bench.py $B 20 2>/dev/null | tail -1
    done
  done
done
