#!/bin/bash
# End-of-round collection on one MI355X (repo root, under gpurun):
#   bench lines (C4 configs[1] and chess configs[4] shard, CPU baselines),
#   C4 rocprofv3 trace + PMC (collect_r1.sh), chess trace + PMC traffic.
set -e
R=$PWD
OUT=$R/gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err
timeout -k 10 400 python3 bench.py --game chess > $OUT/bench_chess.json 2> $OUT/bench_chess.err
bash profiles/collect_r1.sh > $OUT/collect_r1.log 2>&1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/chess_trace -o run --output-format csv -- \
  python3 $R/bench.py --game chess --warmup 1 --steps 1 --no-cpu-baseline > $OUT/chess_trace.json 2> $OUT/chess_trace.err)
bash profiles/pmc_chess_traffic.sh 256 > $OUT/pmc_chess.log 2>&1
echo done
