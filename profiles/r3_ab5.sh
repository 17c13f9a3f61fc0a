#!/bin/bash
# round 3 A/B 5: single tap body with wave-uniform branch skips (br) vs three compiled tap bodies (base)
set -o pipefail
out=gpurun_out/r3_ab5
mkdir -p $out
AZ_LIB_PATH=$PWD/profiles/ab_libs/br/libaz.so timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "tower or keras or batch_invariant or replays" \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for v in base br base br; do
  bash profiles/tower_ab.sh run $v 2>&1 | grep -v amdgpu.ids | tee -a $out/times.txt || exit 1
done
i=0
for v in base br base br; do
  i=$((i+1))
  if [ $v = base ]; then lib=custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=profiles/ab_libs/$v/libaz.so; fi
  AZ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-cache-window > $out/b${v}_$i.json 2> $out/b${v}_$i.err || { tail -5 $out/b${v}_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$out/b${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', d['value'], d['ms_per_step'], 'tower', r['avg_launch_ms'], 'frac', r['frac'], 'iso', r['isolated']['avg_launch_ms'], 'busy_union', r['busy_union']['frac'])" | tee -a $out/bench.txt
done
