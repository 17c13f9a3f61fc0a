#!/bin/bash
# Round-5 GPU session N: the product build's profiles and bench lines --
# kernel trace + PMC (profiles/r5/collect_pmc.sh), the PMC files put where
# bench.py reads them (profiles/r5/, matched by build id), then every config line.
set -o pipefail
bash profiles/r5/collect_pmc.sh > gpurun_out/collect_pmc.log 2>&1 || { tail -20 gpurun_out/collect_pmc.log; exit 1; }
tail -12 gpurun_out/collect_pmc.log
cp gpurun_out/prof_r5/pmc_tower.json gpurun_out/prof_r5/pmc_chess.json profiles/r5/ || exit 1
bash profiles/r5/run_configs.sh
