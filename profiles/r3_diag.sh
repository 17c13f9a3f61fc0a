#!/bin/bash
# round 3: tower K-loop diagnostics with the slot plan (wrong outputs by
# design): no weight stream (nob), no activation reads (noa), neither (noab)
set -o pipefail
out=gpurun_out/r3_diag
mkdir -p $out
for v in stamps st_nob st_noa st_noab; do
  AZ_LIB_PATH=$PWD/profiles/ab_libs/$v/libaz.so timeout -k 10 120 python profiles/tower_stamps.py 4096 2>&1 | grep -v amdgpu.ids > $out/$v.txt || exit 1
  echo "== $v"; grep -E "total|b1.c1loop|b1.c2loop|wave [04]" $out/$v.txt
done
