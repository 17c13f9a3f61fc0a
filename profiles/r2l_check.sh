#!/bin/bash
# GPU suite, select stamps (network) on the diagnostic build, then in-bench A/B
set -o pipefail
mkdir -p gpurun_out/r2g gpurun_out/sel_stamps
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2g/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2g/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2g/gpu_tests.log
AZ_LIB_PATH=$PWD/profiles/ab_libs/selst/libaz.so timeout -k 10 300 python3 profiles/sel_stamps.py > gpurun_out/sel_stamps/network.txt 2>&1 || { tail gpurun_out/sel_stamps/network.txt; exit 1; }
cat gpurun_out/sel_stamps/network.txt
[ $# -gt 0 ] && bash profiles/ab_libs.sh "$@"
