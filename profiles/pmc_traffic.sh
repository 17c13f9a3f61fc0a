#!/bin/bash
# HBM traffic of the conv kernels per board (rocprofv3 FETCH_SIZE and
# WRITE_SIZE in separate passes, az_forward microbenchmark at B boards),
# written to profiles/<round>/pmc_conv_traffic.json for bench.py's roofline.traffic.
# Usage (repo root, under gpurun): bash profiles/pmc_traffic.sh [B] [round]
set -e
R=$PWD
B=${1:-4096}
RND=${2:-r2}
OUT=$R/gpurun_out/pmc_traffic
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for algo in 0 1; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$algo -o run --output-format csv -- \
    python3 $R/profiles/conv_bench.py $B 2 $algo > $OUT/fetch_$algo.txt 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$algo -o run --output-format csv -- \
    python3 $R/profiles/conv_bench.py $B 2 $algo > $OUT/write_$algo.txt 2>&1
done
cd $R
python3 profiles/pmc_traffic.py $OUT $B > $OUT/pmc_conv_traffic.json  # gpurun only brings gpurun_out/ back
cat $OUT/pmc_conv_traffic.json
