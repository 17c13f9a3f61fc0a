#!/bin/bash
# Round-6 bench lines for BASELINE.json's configs on one MI355X (repo root, under gpurun):
# configs[1] (the headline, with the CPU legs), configs[2] 9x9, configs[3] at its 2-GPU shard
# size (16384 games per GPU, S=400), configs[4] chess at its 8-GPU shard size (256 games),
# opening and past 40 untimed moves.  ONLY="c4 c5 ..." picks a subset.
set -o pipefail
T=${TAG:-r6}
OUT=gpurun_out/r6/configs_$T
mkdir -p $OUT
want() { [ -z "$ONLY" ] || [[ " $ONLY " == *" $1 "* ]]; }
if want c4; then
  timeout -k 10 500 python3 -u bench.py > $OUT/c4.json 2> $OUT/c4.err || exit 1
fi
if want c5; then
  timeout -k 10 600 python3 -u bench.py --height 9 --width 9 --n 5 --sims 200 --slots 8192 --steps 10 --warmup 30 \
    --no-cpu-baseline > $OUT/c5_9x9.json 2> $OUT/c5_9x9.err || exit 1
fi
if want s400; then
  timeout -k 10 600 python3 -u bench.py --sims 400 --slots 16384 --steps 10 --warmup 30 --no-cpu-baseline \
    > $OUT/s400_16k.json 2> $OUT/s400_16k.err || exit 1
fi
if want chess; then
  timeout -k 10 400 python3 -u bench.py --game chess --no-cpu-baseline > $OUT/chess.json 2> $OUT/chess.err || exit 1
fi
if want chess_mid; then
  timeout -k 10 500 python3 -u bench.py --game chess --warmup 40 --no-cpu-baseline > $OUT/chess_mid.json \
    2> $OUT/chess_mid.err || exit 1
fi
for f in $OUT/*.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
c=d.get('transposition_cache') or d.get('cache') or {}
print('$f', d['value'], d['unit'], 'ms/step', d.get('ms_per_step'), 'frac', r['frac'], 'bpl', r.get('boards_per_launch'),
      'mfma_busy', r.get('mfma_busy'), 'traffic', r.get('traffic'), 'hit', c.get('hit_rate'))"; done
