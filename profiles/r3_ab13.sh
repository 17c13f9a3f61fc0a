#!/bin/bash
# round 3 A/B 13: static priority for the younger half, no per-k-step turn (sprio) vs base
set -o pipefail
out=gpurun_out/r3_ab13
mkdir -p $out
for v in sprio; do
  AZ_LIB_PATH=$PWD/profiles/ab_libs/$v/libaz.so timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "tower or keras or batch_invariant" \
    > $out/tests_$v.log 2>&1 || { tail -30 $out/tests_$v.log; exit 1; }
  tail -1 $out/tests_$v.log
done
i=0
for v in base sprio base sprio; do
  i=$((i+1))
  if [ $v = base ]; then lib=custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=profiles/ab_libs/$v/libaz.so; fi
  AZ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-cache-window > $out/b${v}_$i.json 2> $out/b${v}_$i.err || { tail -5 $out/b${v}_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$out/b${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', d['value'], d['ms_per_step'], 'tower', r['avg_launch_ms'], 'frac', r['frac'], 'iso', r['isolated']['avg_launch_ms'], 'busy_union', r['busy_union']['frac'])" | tee -a $out/bench.txt
done
AZ_LIB_PATH=$PWD/profiles/ab_libs/st_sprio/libaz.so timeout -k 10 120 python profiles/tower_stamps.py 4096 2>&1 | grep -v amdgpu.ids | grep -E "B=|wave [0-7]|heads1x1|end " | tee -a $out/stamps.txt
