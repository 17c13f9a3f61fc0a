#!/bin/bash
# Round-5 GPU session I: round 4's final tree (git 9278fe6, built in
# profiles/ab_trees/r4) against this tree on ONE box: the isolated forward
# (conv_bench at the bench batch and at 4096) and the default bench, alternating.
set -o pipefail
out=gpurun_out/r5i
mkdir -p $out
R4=profiles/ab_trees/r4
for r in 1 2; do
  timeout -k 10 120 python3 $R4/profiles/conv_bench.py 684 20 0 2>&1 | tail -1 | sed 's/^/r4 /' | tee -a $out/iso.txt || exit 1
  timeout -k 10 120 python3 profiles/conv_bench.py 684 20 0 2>&1 | tail -1 | sed 's/^/r5 /' | tee -a $out/iso.txt || exit 1
  timeout -k 10 120 python3 $R4/profiles/conv_bench.py 4096 10 0 2>&1 | tail -1 | sed 's/^/r4 /' | tee -a $out/iso.txt || exit 1
  timeout -k 10 120 python3 profiles/conv_bench.py 4096 10 0 2>&1 | tail -1 | sed 's/^/r5 /' | tee -a $out/iso.txt || exit 1
done
for r in 1 2; do
  for t in r4 r5; do
    if [ $t = r4 ]; then b=$R4/bench.py; else b=bench.py; fi
    timeout -k 10 300 python3 $b --no-cpu-baseline > $out/bench_$t.json 2> $out/bench_$t.err || { tail -5 $out/bench_$t.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$out/bench_$t.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$t', d['value'], 'ms/step', round(d['ms_per_step'],2), 'launch_ms', r.get('avg_launch_ms'), 'iso', (r.get('isolated') or {}).get('avg_launch_ms'), 'boards', r.get('boards_per_launch'), flush=True)" | tee -a $out/bench.txt
  done
done
