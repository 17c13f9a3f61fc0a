#!/bin/bash
# rocprofv3 kernel stats + per-stream chain of the chess bench (one lane)
set -e
R=$PWD; OUT=$R/gpurun_out/chess_trace; mkdir -p $OUT; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- \
  python3 $R/bench.py --game chess --steps 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err)
T=$(find $OUT/t -name "*kernel_trace.csv" | head -1)
python3 profiles/chain.py $T 1.0 0.3 > $OUT/chain.txt
find $OUT/t -name "*kernel_trace.csv" -delete
python3 - $(find $OUT/t -name "*kernel_stats.csv" | head -1) <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:16]:
    print("  %-44s %7s calls avg %8.1f us  %5.1f%%" % (r["Name"].split("(")[0][-44:], r["Calls"], float(r["AverageNs"])/1e3, float(r["Percentage"])))
PY
cat $OUT/chain.txt
