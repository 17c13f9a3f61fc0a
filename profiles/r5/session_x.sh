#!/bin/bash
# configs[4] chess games to their end (800 sims, synthetic bitwise vs the oracle; network by the rules + replay),
# then chess lanes 2/3/4 with 8 hardware queues
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_chess_fullgame_gpu.py -x -v --durations=0 --timeout 500 --timeout-method thread > gpurun_out/x_tests.log 2>&1; rc=$?; tail -15 gpurun_out/x_tests.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do for l in 2 3 4; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --game chess --lanes $l > gpurun_out/x_l$l.json 2> gpurun_out/x_l$l.err || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/x_l$l.json').read().strip().splitlines()[-1]); r=d['roofline']
print('lanes $l', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],1), 'frac', r['frac'], 'union', r.get('busy_union',{}).get('frac'), 'launch_ms', r.get('avg_launch_ms'), flush=True)" | tee -a gpurun_out/x_lanes.txt
done; done
