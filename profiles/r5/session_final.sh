#!/bin/bash
# Round-5 final build: kernel trace + PMC (collect_pmc.sh), the PMC files put
# where bench.py reads them (matched by build id), then every config line
set -o pipefail
TAG=_final bash profiles/r5/collect_pmc.sh > gpurun_out/collect_final.log 2>&1 || { tail -20 gpurun_out/collect_final.log; exit 1; }
tail -5 gpurun_out/collect_final.log
cp gpurun_out/prof_r5_final/pmc_tower.json gpurun_out/prof_r5_final/pmc_chess.json profiles/r5/ || exit 1
TAG=${CTAG:-r5final2} bash profiles/r5/run_configs.sh
