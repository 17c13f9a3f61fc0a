#!/bin/bash
# Round-5 GPU session G: where the Connect-4 in-bench tower launch went
# (r4 0.195 ms, this round 0.229-0.242 ms on two boxes): the isolated
# forward at the bench's batch on the product and the compiled-loop build,
# then a kernel trace of a short bench window (per-kernel averages vs r4's
# summary_r4k.md).
set -o pipefail
out=gpurun_out/r5g
mkdir -p $out
for v in base kloop_cc base kloop_cc; do
  if [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
  AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 684 20 0 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt
  AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 4096 10 0 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt
done
R=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --no-cpu-baseline --no-cache-window > $R/$out/bench_trace.json 2> $R/$out/bench_trace.err || exit 1
cd $R
python3 profiles/summarize.py $out r5 > $out/summary.md 2>&1
find $out -name "*kernel_trace.csv" -size +20M -delete
head -25 $out/summary.md
