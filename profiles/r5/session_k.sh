#!/bin/bash
# Round-5 GPU session K: the term-major assembly K loop (variants/term.py)
# against the block-major product and the compiled loop -- tower parity on
# the term build first, then the isolated forward and the bench, alternating.
set -o pipefail
out=gpurun_out/r5k
mkdir -p $out
AZ_LIB_PATH=$PWD/profiles/ab_libs/term/libaz.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py \
  tests/test_chess_tree_gpu.py -x -q -k "forward or network or tower" --timeout 200 --timeout-method thread \
  > $out/term_tests.log 2>&1 || { tail -20 $out/term_tests.log; exit 1; }
tail -2 $out/term_tests.log
for r in 1 2; do
  for v in base term kloop_cc; do
    if [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 684 20 0 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt || exit 1
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 4096 10 0 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt || exit 1
  done
done
bash profiles/r5/ab_bench.sh 2 "" base term kloop_cc 2>&1 | tee $out/ab.txt
bash profiles/r5/ab_bench.sh 1 "--game chess" base term 2>&1 | tee $out/ab_chess.txt
