#!/bin/bash
# Round-5 GPU session S: two Connect-4 workgroups per CU (variants/occ4.py:
# 96-row in-place tiles of two boards, <= 80 KB LDS, 4 waves per SIMD)
# against the product (128-row double-buffered tiles, one per CU).
set -o pipefail
out=gpurun_out/r5s
mkdir -p $out
AZ_LIB_PATH=$PWD/profiles/ab_libs/occ4/libaz.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q \
  -k "forward or network or tower" --timeout 200 --timeout-method thread > $out/occ4_tests.log 2>&1 \
  || { tail -20 $out/occ4_tests.log; exit 1; }
tail -2 $out/occ4_tests.log
for r in 1 2; do
  for v in base occ4; do
    if [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 456 20 0 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt || exit 1
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 4096 10 0 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt || exit 1
  done
done
bash profiles/r5/ab_bench.sh 2 "" base occ4 2>&1 | tee $out/ab.txt
bash profiles/r5/ab_bench.sh 1 "--sims 400 --slots 16384 --steps 10 --warmup 30" base occ4 2>&1 | tee $out/ab_s400.txt
