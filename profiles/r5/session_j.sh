#!/bin/bash
# Round-5 GPU session J: is the Connect-4 difference to round 4's tree the
# games themselves?  This tree with the games' streams as round 4 started
# them (--rng-skip 0) against the reference's offset (default) and round 4's tree.
set -o pipefail
out=gpurun_out/r5j
mkdir -p $out
R4=profiles/ab_trees/r4
for r in 1 2; do
  for t in r4 skip0 r5; do
    case $t in r4) cmd="$R4/bench.py";; skip0) cmd="bench.py --rng-skip 0";; r5) cmd="bench.py";; esac
    timeout -k 10 300 python3 $cmd --no-cpu-baseline > $out/bench_$t.json 2> $out/bench_$t.err || { tail -5 $out/bench_$t.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$out/bench_$t.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$t', d['value'], 'ms/step', round(d['ms_per_step'],2), 'launch_ms', r.get('avg_launch_ms'), 'iso', (r.get('isolated') or {}).get('avg_launch_ms'), 'boards', r.get('boards_per_launch'), 'hit', d.get('transposition_cache',{}).get('hit_rate'), 'depth', d.get('roofline_tree',{}).get('mean_depth'), flush=True)" | tee -a $out/bench.txt
  done
done
