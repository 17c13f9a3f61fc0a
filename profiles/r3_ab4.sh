#!/bin/bash
# round 3 A/B 4: SIMD-pair priority schemes in the tower K loop (isolated
# forward times), stamps of two of them
set -o pipefail
out=gpurun_out/r3_ab4
mkdir -p $out
for v in base noalt bal alt1 alt2 prio base; do
  bash profiles/tower_ab.sh run $v 2>&1 | grep -v amdgpu.ids | tee -a $out/times.txt || exit 1
done
for v in st_noalt st_bal; do
  AZ_LIB_PATH=$PWD/profiles/ab_libs/$v/libaz.so timeout -k 10 120 python profiles/tower_stamps.py 4096 2>&1 | grep -v amdgpu.ids > $out/$v.txt || exit 1
  grep -E "total|wave [0-7]" $out/$v.txt
done
