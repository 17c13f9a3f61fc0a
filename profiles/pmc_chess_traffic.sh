#!/bin/bash
# HBM traffic of the chess network's Winograd convs per board (rocprofv3
# FETCH_SIZE and WRITE_SIZE in separate passes, az_chess_forward at B boards)
# -> profiles/r1/pmc_chess_traffic.json (bench.py --game chess roofline.traffic).
# Usage (repo root, under gpurun): bash profiles/pmc_chess_traffic.sh [B]
set -e
R=$PWD
B=${1:-256}
OUT=$R/gpurun_out/pmc_chess_traffic
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_0 -o run --output-format csv -- \
  python3 $R/profiles/chess_conv_bench.py $B 2 > $OUT/fetch_0.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_0 -o run --output-format csv -- \
  python3 $R/profiles/chess_conv_bench.py $B 2 > $OUT/write_0.txt 2>&1
cd $R
python3 profiles/pmc_traffic.py $OUT $B --only 0 > $OUT/pmc_chess_traffic.json
cat $OUT/pmc_chess_traffic.json
