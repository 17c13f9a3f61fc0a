#!/bin/bash
# the other BASELINE configs + chess on the round-3 build (one MI355X)
set -o pipefail
bash profiles/bench_configs.sh || exit 1
timeout -k 10 300 python bench.py --game chess > gpurun_out/configs/chess.json 2> gpurun_out/configs/chess.err || { tail gpurun_out/configs/chess.err; exit 1; }
for f in s400 s400_32k c5_9x9 chess; do
python3 -c "
import json; d=json.loads(open('gpurun_out/configs/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], d['unit'], 'exp/s', d.get('expansions_per_s'), 'frac', r['frac'], 'hit', (d.get('transposition_cache') or {}).get('hit_rate'))"
done
