#!/bin/bash
# Round-6 final build, call B (repo root, under gpurun): the configs[1]
# headline line with the CPU legs, the window-event placements (tower only /
# select + tower + expand / none; same library), the chess lines (opening and
# past move 40).
set -o pipefail
T=final
OUT=gpurun_out/r6/configs_$T
mkdir -p $OUT
timeout -k 10 500 python3 -u bench.py > $OUT/c4.json 2> $OUT/c4.err || { tail -20 $OUT/c4.err; exit 1; }
tail -c 200 $OUT/c4.json; echo
for ev in 1 tree 0; do
  o=$OUT/ev_$ev.json
  AZ_BENCH_WINDOW_EVENTS=$ev timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window > $o 2> ${o%.json}.err \
    || { tail -5 ${o%.json}.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$o').read().strip().splitlines()[-1]); r=d['roofline']
print('events $ev', d['value'], 'ms/step', d['ms_per_step'], 'tower us', round(r['avg_launch_ms']*1e3,1), flush=True)"
done
ONLY="chess chess_mid" TAG=$T bash profiles/r6/run_configs.sh
