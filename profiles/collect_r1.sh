#!/bin/bash
# rocprofv3 collection for round 1 (run from the repo root under gpurun).
# Pass 1: kernel trace + stats of a short bench.py run (timing; the bench's own
#         HIP-event avg_launch_ms in bench_trace.json must agree with it).
# Pass 2: HBM traffic of the conv kernels (FETCH_SIZE, WRITE_SIZE: separate
#         passes) -> profiles/r1/pmc_conv_traffic.json (pmc_traffic.sh).
# Pass 3: SQ counters (MFMA busy, wave stall breakdown) of the conv kernels.
set -e
R=$PWD
OUT=$R/gpurun_out/prof_r1
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 20 --no-cpu-baseline --no-cache-window > $OUT/bench_trace.json 2> $OUT/bench_trace.err)
bash profiles/pmc_traffic.sh 4096 > $OUT/pmc_traffic.log 2>&1
bash profiles/pmc_conv.sh 4096 0 > $OUT/pmc_conv.log 2>&1
python3 profiles/summarize.py $OUT > $OUT/summary.md
cat $OUT/summary.md
