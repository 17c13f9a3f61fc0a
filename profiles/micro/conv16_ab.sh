#!/bin/bash
# A/B builds of conv16_kernel (macro variants) on the sweep's C4 / chess shapes,
# plus PMC counters for the default build at the self-play batch.
set -o pipefail
out=${1:-gpurun_out/c16ab}
mkdir -p "$out"
for v in "-DAZ_C16_PF=2" "-DAZ_C16_PF=2 -DAZ_C16_APF=1"; do
  tag=$(echo "$v" | tr -dc 'A-Z0-9_=' )
  hipcc --offload-arch=gfx950 -O3 -std=c++17 $v profiles/micro/conv16_bench.cpp -o /tmp/c16_$$ || exit 1
  for cfg in "870 6 7 1" "4096 6 7 1" "256 8 8 1"; do
    for mode in 0 1; do
      echo -n "$tag " >> "$out/ab.txt"
      timeout -k 5 60 /tmp/c16_$$ $cfg $mode 50 >> "$out/ab.txt" || exit 1
    done
  done
done
cat "$out/ab.txt"
cd /tmp && export TMPDIR=/tmp
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT TCP_TCC_READ_REQ_sum"; do
  timeout -s KILL 60 rocprofv3 --pmc $pmc -d $OLDPWD/$out/pmc -o p$(echo $pmc | wc -c) -- $OLDPWD/profiles/micro/conv16_bench 4096 6 7 1 0 20 > /dev/null || exit 1
done
