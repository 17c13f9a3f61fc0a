#!/bin/bash
# round 3 A/B 10: the generalized slot plan (top | bottom for one 9x9 board
# per 96-row tile): engine GPU tests, configs[2] with AZ_TOWER_PLAN=1/0, C4 bench
set -o pipefail
out=gpurun_out/r3_ab10
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for p in 1 0 1 0; do
  AZ_TOWER_PLAN=$p timeout -k 10 400 python bench.py --height 9 --width 9 --n 5 --sims 200 --slots 8192 --steps 10 --warmup 30 --no-cpu-baseline --no-cache-window > $out/c5_$p.json 2> $out/c5_$p.err || { tail -5 $out/c5_$p.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$out/c5_$p.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c5 plan $p', d['value'], d['expansions_per_s'], 'tower', r['avg_launch_ms'], 'frac', r['frac'], 'issued', r['issued']['flop_per_board'])" | tee -a $out/bench.txt
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-cache-window > $out/c4.json 2> $out/c4.err || { tail -5 $out/c4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$out/c4.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c4', d['value'], 'frac', r['frac'], 'issued', r['issued']['flop_per_board'])" | tee -a $out/bench.txt
