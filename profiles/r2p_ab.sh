#!/bin/bash
# GPU suite on the current build, then in-bench A/B of the heads/stem rewrite
# (old = HEAD before it, base = register-weight heads + 64-channel stem blocks,
# h2 = base with the 128-channel stem blocks).  Usage: bash profiles/r2p_ab.sh
set -o pipefail
out=gpurun_out/r2p
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
bash profiles/ab_libs.sh old base h2 old base h2
