#!/bin/bash
# Round-5 GPU session T: the select descent touching the next level's edges
# (LDS-DMA cache touches) -- tree parity first (fixtures, replays), the
# select stamps of the touch build, then in-bench A/B against no touches.
set -o pipefail
out=gpurun_out/r5t
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_api_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -2 $out/tests.log
AZ_LIB_PATH=$PWD/profiles/ab_libs/selst_touch/libaz.so timeout -k 10 240 python3 -u profiles/sel_stamps.py > $out/sel_stamps.txt 2>&1 || exit 1
tail -14 $out/sel_stamps.txt
bash profiles/r5/ab_bench.sh 3 "" base notouch 2>&1 | tee $out/ab.txt
