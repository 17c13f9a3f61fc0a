#!/bin/bash
# rocprofv3 collection for round 1 (run from the repo root under gpurun).
# Pass 1: kernel trace + stats (timing).  Passes 2-3: HBM traffic counters,
# each in its own run (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
set -e
R=$PWD
OUT=$R/gpurun_out/prof_r1
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 5 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/bench_trace.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_write.json 2> $OUT/bench_write.err
ls -R $OUT | head -40
