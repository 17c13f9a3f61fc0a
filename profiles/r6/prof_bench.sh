#!/bin/bash
# rocprofv3 kernel trace of one bench.py run (repo root, under gpurun):
#   prof_bench.sh TAG [bench.py args]
# keeps the per-kernel stats, the summary (profiles/summarize.py: top kernels,
# occupancy over the trace's last 0.5 s) and the per-stream chain; deletes the
# kernel trace itself (hundreds of MB after a long cache preroll).
set -o pipefail
R=$PWD
TAG=$1; shift
OUT=$R/gpurun_out/r6/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-cache-window "$@" > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit 1
cd $R
tr=$(find $OUT/trace -name '*kernel_trace.csv' | head -1)
python3 profiles/summarize.py $OUT r6 > $OUT/summary.md
python3 profiles/chain.py $tr 0.3 > $OUT/chain.txt || true
find $OUT/trace -name '*kernel_trace.csv' -delete
cat $OUT/summary.md
