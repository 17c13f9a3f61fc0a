#!/bin/bash
# Round-6 final build, call A (repo root, under gpurun): the GPU suite, the
# default bench line, the window-events A/B (every launch vs every 4th), the
# PMC passes and a rocprofv3 kernel trace of the bench -- all for this build.
set -o pipefail
OUT=gpurun_out/r6/final
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 500 python3 -u bench.py > $OUT/c4.json 2> $OUT/c4.err || { tail -20 $OUT/c4.err; exit 1; }
tail -c 300 $OUT/c4.json; echo
for i in 1 2; do
  for ev in 1 4; do
    o=$OUT/ev${ev}_$i.json
    AZ_BENCH_WINDOW_EVENTS=$ev timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window > $o 2> ${o%.json}.err \
      || { tail -5 ${o%.json}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$o').read().strip().splitlines()[-1]); r=d['roofline']
print('events every $ev', d['value'], 'ms/step', d['ms_per_step'], 'tower us', round(r['avg_launch_ms']*1e3,1), 'bpl', r['boards_per_launch'], 'union', r['busy_union']['frac'], flush=True)"
  done
done
TAG=_final bash profiles/r6/collect_pmc.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
bash profiles/r6/prof_bench.sh final > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
head -20 $OUT/prof.log
echo final_a done
