#!/bin/bash
# fused expand+select: GPU parity, then in-bench A/B against the split launches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w_tests.log 2>&1 && tail -3 gpurun_out/w_tests.log &&
bash profiles/r5/ab_bench.sh 3 "" base nofuse:AZ_FUSE_EXPAND=0 2>&1 | tee gpurun_out/w_ab.txt &&
bash profiles/r5/ab_bench.sh 1 "--sims 400 --slots 16384 --steps 10 --warmup 30" base nofuse:AZ_FUSE_EXPAND=0 2>&1 | tee gpurun_out/w_ab_s400.txt
