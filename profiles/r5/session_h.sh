#!/bin/bash
# Round-5 GPU session H: what lengthened the Connect-4 period (r4 29.3 ms per
# move, this round 32.2-32.4 at equal isolated tower time): the bounded
# arenas (--arena-edges bounded vs proof) and the dedup in the select launch
# (variants/dedupk.py: its own launch again), alternating on one box.
set -o pipefail
out=gpurun_out/r5h
mkdir -p $out
for r in 1 2; do
  bash profiles/r5/ab_bench.sh 1 "" base dedupk 2>&1 | tee -a $out/ab.txt || exit 1
  bash profiles/r5/ab_bench.sh 1 "--arena-edges proof" base 2>&1 | sed 's/^base/proof/' | tee -a $out/ab.txt || exit 1
done
