#!/bin/bash
# GPU suite, then in-bench A/B of libaz builds (profiles/ab_libs.sh)
# usage: bash profiles/r2g_check.sh <variant>...
set -o pipefail
mkdir -p gpurun_out/r2g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2g/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2g/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2g/gpu_tests.log
[ $# -gt 0 ] && bash profiles/ab_libs.sh "$@"
