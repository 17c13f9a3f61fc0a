#!/bin/bash
# the GPU suite and smoke() on the final build
set -o pipefail
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_final.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1; rc=$?; tail -3 gpurun_out/smoke_final.log; exit $rc
