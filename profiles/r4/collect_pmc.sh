#!/bin/bash
# Round-4 PMC + trace collection for the benched build (repo root, under gpurun):
#  1. kernel trace + stats of a short bench.py run (its HIP-event avg_launch_ms
#     must agree with rocprof's average for tower16_kernel)
#  2. PMC passes over az_forward at the live lane batch (672 boards): FETCH_SIZE,
#     WRITE_SIZE, then MFMA busy (each its own pass) -> profiles/r4/pmc_tower.json,
#     stamped with the build id bench.py matches
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/prof_r4${TAG:-}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --no-cpu-baseline --no-cache-window > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc/fetch -o run --output-format csv -- \
  python3 $R/profiles/conv_bench.py 672 10 0 > $OUT/pmc_fetch.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc/write -o run --output-format csv -- \
  python3 $R/profiles/conv_bench.py 672 10 0 > $OUT/pmc_write.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $OUT/pmc/sq -o run --output-format csv -- \
  python3 $R/profiles/conv_bench.py 672 10 0 > $OUT/pmc_sq.txt 2>&1 || exit 1
cd $R
python3 profiles/pmc_fold.py $OUT/pmc 672 tower16_kernel tower16 > $OUT/pmc_tower.json || exit 1
python3 profiles/summarize.py $OUT r4 > $OUT/summary.md 2>&1
find $OUT -name "*kernel_trace.csv" -size +20M -delete
cat $OUT/pmc_tower.json
tail -30 $OUT/summary.md
