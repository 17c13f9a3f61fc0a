#!/bin/bash
# Round-5 GPU session F: chess tower regression hunt (r4 108.5 us per
# 128-board launch, this round's first line 166.5): 16 vs 8 waves per
# one-board tile, assembly vs compiled K loop, weight prefetch 1 vs 2;
# chess network parity on the 8-wave form first.
set -o pipefail
out=gpurun_out/r5f
mkdir -p $out
AZ_LIB_PATH=$PWD/profiles/ab_libs/chess8w/libaz.so timeout -k 10 300 python -u -m pytest tests/test_chess_tree_gpu.py \
  tests/test_chess_selfplay_gpu.py -x -q --timeout 200 --timeout-method thread -k network > $out/chess8w_tests.log 2>&1 \
  || { tail -20 $out/chess8w_tests.log; exit 1; }
tail -2 $out/chess8w_tests.log
bash profiles/r5/ab_bench.sh 2 "--game chess" base kloop_cc chess8w chess8w_cc pf1 2>&1 | tee $out/ab_chess.txt
