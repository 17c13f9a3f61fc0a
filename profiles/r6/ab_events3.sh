#!/bin/bash
# The timed window's HIP events (same library, alternating on one box):
# tower launches only (1), select + tower + expand (tree), none (0)
set -o pipefail
OUT=gpurun_out/r6/abe3
mkdir -p $OUT
for i in 1 2; do
  for ev in 1 tree 0; do
    o=$OUT/ev${ev}_$i.json
    AZ_BENCH_WINDOW_EVENTS=$ev timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window > $o 2> ${o%.json}.err \
      || { tail -5 ${o%.json}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$o').read().strip().splitlines()[-1]); r=d['roofline']
print('events $ev', d['value'], 'ms/step', d['ms_per_step'], 'tower us', round(r['avg_launch_ms']*1e3,1), flush=True)"
  done
done
