#!/bin/bash
# kernel trace of a short bench run -> per-stream chain/gap analysis (profiles/chain.py)
set -e
R=$PWD
OUT=$R/gpurun_out/chain
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 12 --no-cpu-baseline --no-cache-window > $OUT/bench.json 2> $OUT/bench.err)
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 profiles/chain.py $T 0.3 0.45 > $OUT/chain.txt   # inside the timed window (12 steps ~ 0.7 s)
python3 profiles/chain.py $T 0.15 0.0 >> $OUT/chain.txt  # the end: tree-timer window, isolated forwards
find $OUT -name "*kernel_trace.csv" -delete
cat $OUT/chain.txt
