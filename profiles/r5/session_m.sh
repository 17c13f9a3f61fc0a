#!/bin/bash
# Round-5 GPU session M: 8 hardware queues + 3 lanes against the default
# (4 queues, 2 lanes), alternating: configs[1] x3, then configs[2] and the
# configs[3] shard once each.
set -o pipefail
out=gpurun_out/r5m
mkdir -p $out
run() {  # tag queues lanes extra-args
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --lanes $3 $4 > $out/$1.json 2> $out/$1.err \
    || { tail -5 $out/$1.err; return 1; }
  python3 -c "
import json
d=json.loads(open('$out/$1.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$1 q$2 l$3', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],2), 'launch_ms', r.get('avg_launch_ms'), 'union', (r.get('busy_union') or {}).get('frac'), flush=True)" | tee -a $out/ab.txt
}
for r in 1 2 3; do
  run c4_q4l2 4 2 "" || exit 1
  run c4_q8l3 8 3 "" || exit 1
  run c4_q8l2 8 2 "" || exit 1
done
C5="--height 9 --width 9 --n 5 --sims 200 --slots 8192 --steps 10 --warmup 30"
run c5_q4l2 4 2 "$C5" || exit 1
run c5_q8l3 8 3 "$C5" || exit 1
S4="--sims 400 --slots 16384 --steps 10 --warmup 30"
run s4_q4l2 4 2 "$S4" || exit 1
run s4_q8l3 8 3 "$S4" || exit 1
