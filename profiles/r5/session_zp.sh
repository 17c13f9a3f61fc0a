#!/bin/bash
# chess chain: policy dense in the tower tail (no dense launch);
# chess GPU tests, then in-bench A/B against the round-5 final build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_chess_selfplay_gpu.py tests/test_chess_gpu.py tests/test_chess_tree_gpu.py tests/test_chess_fullgame_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/zp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/zp_tests.log; [ $rc = 0 ] || exit $rc
bash profiles/r5/ab_bench.sh 3 "--game chess" base chain6 2>&1 | tee gpurun_out/zp_ab.txt
