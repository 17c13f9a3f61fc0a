#!/bin/bash
# Round-5 GPU session V: chess's one-board tiles in 4 waves (one per SIMD,
# variants/chess1w.py) against 8 -- chess parity on the variant, the
# isolated chess forward, then chess bench A/B.
set -o pipefail
out=gpurun_out/r5v
mkdir -p $out
AZ_LIB_PATH=$PWD/profiles/ab_libs/chess1w/libaz.so timeout -k 10 300 python -u -m pytest tests/test_chess_tree_gpu.py \
  tests/test_chess_selfplay_gpu.py -x -q --timeout 200 --timeout-method thread > $out/chess1w_tests.log 2>&1 \
  || { tail -20 $out/chess1w_tests.log; exit 1; }
tail -2 $out/chess1w_tests.log
for r in 1 2; do
  for v in base chess1w; do
    if [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/chess_conv_bench.py 128 20 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt || exit 1
  done
done
bash profiles/r5/ab_bench.sh 2 "--game chess" base chess1w 2>&1 | tee $out/ab.txt
