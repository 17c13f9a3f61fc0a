#!/bin/bash
# Round-6 last build (the simulation-tag wrap guard on top of d0e3b8e6), repo
# root under gpurun: the GPU suite, its PMC passes, the configs[1] line (which
# reads them) and the chess opening line.
set -o pipefail
OUT=gpurun_out/r6/final_d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
TAG=_d bash profiles/r6/collect_pmc.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
cp gpurun_out/r6/pmc_d/pmc_tower.json profiles/r6/pmc_tower.json && cp gpurun_out/r6/pmc_d/pmc_chess.json profiles/r6/pmc_chess.json
ONLY="c4 chess" TAG=d bash profiles/r6/run_configs.sh
