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
