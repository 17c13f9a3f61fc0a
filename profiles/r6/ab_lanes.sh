#!/bin/bash
# configs[1] games/s against the lane count with the LRU 2^26 cache (round 6):
# the towers shrank to ~120 boards per lane launch, so each lane is a
# latency-bound chain (tower -> select -> expand) and more lanes may fill CUs.
set -o pipefail
mkdir -p gpurun_out/r6
export GPU_MAX_HW_QUEUES=${Q:-16}
for L in "$@"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window --lanes $L > gpurun_out/r6/lanes_$L.json 2> gpurun_out/r6/lanes_$L.err || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6/lanes_$L.json').read().strip().splitlines()[-1])
print('lanes', d['lanes'], 'q', d['hw_queues'], 'games/s', d['value'], 'ms/step', d['ms_per_step'], 'hit', d['transposition_cache']['hit_rate'], 'tower us', round(d['roofline']['avg_launch_ms']*1e3,1), 'boards/launch', d['roofline'].get('boards_per_launch'), 'union', d['roofline'].get('busy_union'))"
done
