#!/bin/bash
# SQ / LDS counters of tower16_kernel over an isolated forward loop (profiles/tower_time.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_tower
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_tower/p$i -o p$i --output-format csv -- python3 $R/profiles/tower_time.py pmc > $R/gpurun_out/pmc_tower/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc_tower/p$i.log; exit 1; }
done
python3 $R/profiles/pmc_summary.py $R/gpurun_out/pmc_tower tower16 2>&1 | tail -30
