#!/bin/bash
# Round-5 GPU session E: the tests session A failed (chess network paths:
# the stem's 2-k-step groups had prefetched the next tap from a wrong
# soffset; the tree-API fixtures' model-construction draws), then the rest.
set -o pipefail
out=gpurun_out/r5e
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_chess_selfplay_gpu.py tests/test_chess_tree_gpu.py tests/test_engine_gpu.py \
  tests/test_fullsize_gpu.py -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider -k "chess or tree_api" \
  > $out/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $out/gpu_tests.log | tail -3
grep -E "FAILED" $out/gpu_tests.log | head -20
exit $rc
