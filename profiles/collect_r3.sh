#!/bin/bash
# rocprofv3 collection for round 3 (repo root, under gpurun); results in
# gpurun_out/prof_r3, the summary copied to profiles/r3 afterwards.
#  1. kernel trace + stats of a short bench.py run (its HIP-event
#     avg_launch_ms must agree with rocprof's average for tower16_kernel)
#  2. HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of the forward's
#     kernels: C4 tower / direct / per-layer at B = 672 (the live lane batch)
#     and the chess per-layer fp16x2 convs at B = 128 -> pmc json files
#  3. SQ counters of the tower at the live batch
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/prof_r3
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --no-cpu-baseline --no-cache-window > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit 1
for algo in 0 1 2; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/traffic/fetch_$algo -o run --output-format csv -- \
    python3 $R/profiles/conv_bench.py 672 3 $algo > $OUT/traffic_f$algo.txt 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/traffic/write_$algo -o run --output-format csv -- \
    python3 $R/profiles/conv_bench.py 672 3 $algo > $OUT/traffic_w$algo.txt 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/chess_traffic/fetch_0 -o run --output-format csv -- \
  python3 $R/profiles/chess_conv_bench.py 128 2 > $OUT/chess_f.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/chess_traffic/write_0 -o run --output-format csv -- \
  python3 $R/profiles/chess_conv_bench.py 128 2 > $OUT/chess_w.txt 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/sq/p$i -o run --output-format csv -- \
    python3 $R/profiles/conv_bench.py 672 5 0 > $OUT/sq_$i.txt 2>&1 || exit 1
done
cd $R
python3 profiles/pmc_traffic.py $OUT/traffic 672 > $OUT/pmc_conv_traffic.json
python3 profiles/pmc_traffic.py $OUT/chess_traffic 128 --only 0 --chess > $OUT/pmc_chess_traffic.json
mkdir -p $R/profiles/r3 && cp $OUT/pmc_conv_traffic.json $OUT/pmc_chess_traffic.json $R/profiles/r3/
python3 profiles/summarize.py $OUT r3 > $OUT/summary.md
python3 profiles/pmc_summary.py $OUT/sq tower16 >> $OUT/summary.md
find $OUT -name "*kernel_trace.csv" -size +20M -delete
cat $OUT/summary.md
