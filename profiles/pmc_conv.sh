#!/bin/bash
# SQ counters for the conv kernels (az_forward microbenchmark, B boards).
# Usage (repo root, under gpurun): bash profiles/pmc_conv.sh [B] [algo]
set -e
R=$PWD
B=${1:-4096}
A=${2:-0}
OUT=$R/gpurun_out/pmc_conv_${B}_${A}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS -d $OUT/sq -o run --output-format csv -- \
  python3 $R/profiles/conv_bench.py $B 3 $A > $OUT/bench.txt 2> $OUT/err.txt
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/grbm -o run --output-format csv -- \
  python3 $R/profiles/conv_bench.py $B 3 $A >> $OUT/bench.txt 2>> $OUT/err.txt
find $OUT -name "*.csv" | head
