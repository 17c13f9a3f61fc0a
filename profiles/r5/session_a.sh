#!/bin/bash
# Round-5 GPU session A: the whole GPU suite on the product build (the
# assembly K loop, 192-row 9x9 tiles, a8 noise tests, chess to termination).
set -o pipefail
out=gpurun_out/r5a
mkdir -p $out
timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > $out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $out/gpu_tests.log | tail -5
tail -15 $out/gpu_tests.log
exit $rc
