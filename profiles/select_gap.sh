#!/bin/bash
# where the per-simulation gap before select_group comes from: host enqueue
# cost of a move, then kernel traces of the bench with 1 and 2 lanes
set -e
R=$PWD
OUT=$R/gpurun_out/select_gap
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python3 profiles/host_enqueue.py > $OUT/host_enqueue.txt 2>&1
cat $OUT/host_enqueue.txt
for L in 2 1; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace$L -o run --output-format csv -- \
    python3 $R/bench.py --steps 12 --lanes $L --no-cpu-baseline --no-cache-window > $OUT/bench$L.json 2> $OUT/bench$L.err)
  T=$(find $OUT/trace$L -name "*kernel_trace.csv" | head -1)
  python3 profiles/chain.py $T 0.3 0.45 > $OUT/chain$L.txt
  gzip -c $T > $OUT/kt$L.csv.gz && find $OUT/trace$L -name "*kernel_trace.csv" -delete
  cat $OUT/chain$L.txt
done
