#!/bin/bash
# Round-6 diagnostics of the simulation chain (repo root, under gpurun):
#  - kernel trace of bench.py with the cache inserts in a launch of their own
#    (variants/splitins.py: times the expand half and the insert half apart)
#  - the 96-row tile's phase clocks at 122 boards (variants/stamps.py)
#  - the select launch's per-slot phase stamps (variants/selst.py)
set -o pipefail
OUT=gpurun_out/r6/diag1
mkdir -p $OUT
AZ_LIB_PATH=$PWD/profiles/ab_libs/splitins/libaz.so bash profiles/r6/prof_bench.sh splitins > $OUT/prof_splitins.log 2>&1 \
  || { tail -20 $OUT/prof_splitins.log; exit 1; }
head -16 $OUT/prof_splitins.log
BPW=2 AZ_LIB_PATH=$PWD/profiles/ab_libs/stamps/libaz.so timeout -k 10 180 python3 profiles/r6/tower_stamps.py 122 \
  > $OUT/stamps96.txt 2>&1 || { tail -20 $OUT/stamps96.txt; exit 1; }
cat $OUT/stamps96.txt | head -24
AZ_LIB_PATH=$PWD/profiles/ab_libs/selst/libaz.so timeout -k 10 240 python3 profiles/sel_stamps.py \
  > $OUT/sel_stamps.txt 2>&1 || { tail -20 $OUT/sel_stamps.txt; exit 1; }
cat $OUT/sel_stamps.txt
