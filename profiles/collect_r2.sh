#!/bin/bash
# rocprofv3 collection for round 2 (repo root, under gpurun); copy the
# results from gpurun_out/prof_r2 into profiles/r2 afterwards.
# Pass 1: kernel trace + stats of a short bench.py run (its HIP-event
#         avg_launch_ms in bench_trace.json must agree with rocprof's).
# Pass 2: HBM traffic of the conv kernels (FETCH_SIZE, WRITE_SIZE: separate
#         passes, az_forward at B = 4096) -> pmc_conv_traffic.json.
# Pass 3: SQ counters (MFMA busy, stall breakdown, LDS) of the conv kernels
#         at B = 4096 and at the self-play batch (871 boards).
set -e
R=$PWD
OUT=$R/gpurun_out/prof_r2
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --no-cpu-baseline --no-cache-window > $OUT/bench_trace.json 2> $OUT/bench_trace.err)
bash profiles/pmc_traffic.sh 4096 r2 > $OUT/pmc_traffic.log 2>&1
cp $R/gpurun_out/pmc_traffic/pmc_conv_traffic.json $OUT/
mv $R/gpurun_out/pmc_traffic $OUT/
bash profiles/pmc_conv.sh 4096 0 > $OUT/pmc_conv.log 2>&1
bash profiles/pmc_conv.sh 871 0 >> $OUT/pmc_conv.log 2>&1
mv $R/gpurun_out/pmc_conv_4096_0 $R/gpurun_out/pmc_conv_871_0 $OUT/
mkdir -p $R/profiles/r2 && cp $OUT/pmc_conv_traffic.json $R/profiles/r2/
python3 profiles/summarize.py $OUT r2 > $OUT/summary.md
find $OUT -name "*kernel_trace.csv" -delete  # (>64 MiB: gpurun would not copy gpurun_out back)
python3 profiles/pmc_summary.py $OUT/pmc_conv_871_0 conv >> $OUT/summary.md
cat $OUT/summary.md
