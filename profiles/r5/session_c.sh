#!/bin/bash
# Round-5 GPU session C: the assembly K loop (az_kloop_asm.h) -- tower parity
# on the product build, then alternating in-bench A/B against the compiled
# loop (kloop_cc) and the 16-wave tile (nwm4, now on the assembly loop too).
set -o pipefail
out=gpurun_out/r5c
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v -k "forward or network or tower" \
  --timeout 200 --timeout-method thread > $out/tower_tests.log 2>&1 || { tail -30 $out/tower_tests.log; exit 1; }
tail -3 $out/tower_tests.log
bash profiles/r5/ab_bench.sh 2 "" base kloop_cc kloop_pf2 nwm4 2>&1 | tee $out/ab.txt
# configs[2] 9x9: the 192-row in-place tile (two boards per workgroup) against the product
AZ_LIB_PATH=$PWD/profiles/ab_libs/t192/libaz.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q \
  -k "forward_matches or batch_invariant" --timeout 200 --timeout-method thread > $out/t192_tests.log 2>&1 || { tail -20 $out/t192_tests.log; exit 1; }
tail -2 $out/t192_tests.log
bash profiles/r5/ab_bench.sh 1 "--height 9 --width 9 --n 5 --sims 200 --slots 8192 --steps 10 --warmup 30" base t192 2>&1 | tee $out/ab_9x9.txt
