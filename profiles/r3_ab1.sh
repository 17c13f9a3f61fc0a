#!/bin/bash
# round 3 A/B 1: the refactored tower (M-block ring, packed pixel words,
# grouped stem) must stay bit-exact; isolated forward times of one wave per
# SIMD (128 x 32 wave tiles, half the weight stream) against the default
set -o pipefail
mkdir -p gpurun_out/r3_ab1
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3_ab1/tests.log 2>&1 || { tail -30 gpurun_out/r3_ab1/tests.log; exit 1; }
tail -2 gpurun_out/r3_ab1/tests.log
for v in base n1 n1pf2 n1pf3 base; do
  bash profiles/tower_ab.sh run $v 2>&1 | tee -a gpurun_out/r3_ab1/times.txt || exit 1
done
