#!/bin/bash
# chess bench lanes A/B (and a C4 A/B of libaz builds via profiles/ab_libs.sh)
set -o pipefail
mkdir -p gpurun_out/chess_lanes
for l in ${CHESS_LANES:-1 2 1 2}; do
  timeout -k 10 300 python bench.py --game chess --no-cpu-baseline --lanes $l > gpurun_out/chess_lanes/l$l.json 2> gpurun_out/chess_lanes/l$l.err || { tail gpurun_out/chess_lanes/l$l.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/chess_lanes/l$l.json').read().strip().splitlines()[-1]); print('chess lanes $l', d['value'], d['roofline']['avg_launch_ms'])"
done
[ $# -gt 0 ] && bash profiles/ab_libs.sh "$@"
