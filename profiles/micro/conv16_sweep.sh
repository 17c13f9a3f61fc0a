#!/bin/bash
# conv16_kernel check + timing sweep (GPU box): bash profiles/micro/conv16_sweep.sh <out>
set -o pipefail
out=${1:-gpurun_out/conv16_sweep.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
for cfg in "870 6 7" "1000 6 7" "4096 6 7" "256 8 8" "4096 9 9"; do
  for wm in 1 2; do
    for mode in 0 1 2; do
      timeout -k 5 60 ./profiles/micro/conv16_bench $cfg $wm $mode 50 >> "$out" || { echo "FAILED $cfg $wm $mode"; exit 1; }
    done
  done
done
cat "$out"
