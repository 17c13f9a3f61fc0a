#!/bin/bash
# Round-5 GPU session B: hardware queues per process x lanes, Connect-4
# configs[1] (6 runs) and chess configs[4]'s shard at 8 queues (3 runs).
set -o pipefail
bash profiles/r5/ab_queues.sh r5b_q connect_n || exit 1
out=gpurun_out/r5b_q
for lanes in 2 3 4; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 240 python bench.py --game chess --no-cpu-baseline --lanes $lanes \
      > $out/chess_q8_l$lanes.json 2> $out/chess_q8_l$lanes.err || { tail -5 $out/chess_q8_l$lanes.err; exit 1; }
  python - $out/chess_q8_l$lanes.json $lanes <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"chess queues 8 lanes {sys.argv[2]}: {d['value']:.4g} exp/s ms/step {d['ms_per_step']:.1f} frac {d['roofline']['frac']:.4f}", flush=True)
PY
done
