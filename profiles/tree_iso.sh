#!/bin/bash
set -e
R=$PWD; OUT=$R/gpurun_out/tree_iso; mkdir -p $OUT; export TMPDIR=/tmp
for l in 1 2; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/l$l -o run --output-format csv -- python3 $R/profiles/tree_iso.py $l 10 > $OUT/l$l.txt 2>&1)
  cat $OUT/l$l.txt
  find $OUT/l$l -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \; | head -12
  find $OUT/l$l -name "*kernel_trace.csv" -delete
done
