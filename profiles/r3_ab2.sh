#!/bin/bash
# round 3 A/B 2: the tower slot plan (border blocks skip the taps past their
# edge) -- engine GPU tests (bitwise vs natural order), isolated forward
# times and in-bench games/s with AZ_TOWER_PLAN=1/0 alternating
set -o pipefail
out=gpurun_out/r3_ab2
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for p in 1 0 1 0; do
  AZ_TOWER_PLAN=$p timeout -k 10 120 python profiles/tower_time.py plan$p 2>&1 | grep -v amdgpu.ids | tee -a $out/times.txt || exit 1
done
i=0
for p in 1 0 1 0; do
  i=$((i+1))
  AZ_TOWER_PLAN=$p timeout -k 10 300 python bench.py --no-cpu-baseline --no-cache-window > $out/b${p}_$i.json 2> $out/b${p}_$i.err || { tail -5 $out/b${p}_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$out/b${p}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']
print('plan $p', d['value'], d['ms_per_step'], 'tower', r['avg_launch_ms'], 'boards', r['boards_per_launch'], 'frac', r['frac'], 'iso', r['isolated']['avg_launch_ms'], 'busy_union', r['busy_union']['frac'], 'hit', d['transposition_cache']['hit_rate'])" | tee -a $out/bench.txt
done
