#!/bin/bash
# Round-5 GPU session D: bench lines on the product build (configs[1] with
# the CPU legs, configs[2] 9x9, chess configs[4] shard opening and mid-game),
# then A/B: the compiled K loop (kloop_cc) and Connect-4 on 192-row tiles
# (c4t192) at configs[1] and at the configs[3] shard (16384 games, S=400).
set -o pipefail
out=gpurun_out/r5d
mkdir -p $out
timeout -k 10 420 python3 -u bench.py > $out/c4.json 2> $out/c4.err || { tail -5 $out/c4.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --height 9 --width 9 --n 5 --sims 200 --slots 8192 --steps 10 --warmup 30 \
  --no-cpu-baseline > $out/c5_9x9.json 2> $out/c5_9x9.err || { tail -5 $out/c5_9x9.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --game chess --no-cpu-baseline > $out/chess.json 2> $out/chess.err || { tail -5 $out/chess.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --game chess --warmup 40 --no-cpu-baseline > $out/chess_mid.json 2> $out/chess_mid.err || { tail -5 $out/chess_mid.err; exit 1; }
for f in $out/*.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],1), 'frac', r['frac'], 'union', (r.get('busy_union') or {}).get('frac'), 'launch_ms', r.get('avg_launch_ms'))"; done
bash profiles/r5/ab_bench.sh 2 "" base kloop_cc c4t192 2>&1 | tee $out/ab_c4.txt
bash profiles/r5/ab_bench.sh 1 "--sims 400 --slots 16384 --steps 10 --warmup 30" base c4t192 2>&1 | tee $out/ab_s400.txt
