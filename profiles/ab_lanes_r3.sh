#!/bin/bash
# in-bench lanes A/B on the current build
set -o pipefail
mkdir -p gpurun_out/lanes_r3
for L in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-cache-window --lanes $L > gpurun_out/lanes_r3/l$L.json 2> gpurun_out/lanes_r3/l$L.err || { tail -5 gpurun_out/lanes_r3/l$L.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/lanes_r3/l$L.json').read().strip().splitlines()[-1]); r=d['roofline']
print('lanes $L', d['value'], d['ms_per_step'], 'tower', r['avg_launch_ms'], 'boards', r['boards_per_launch'], 'frac', r['frac'], 'iso', r['isolated']['avg_launch_ms'], 'busy_union', r['busy_union']['frac'])"
done
