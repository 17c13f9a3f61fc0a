#!/bin/bash
# A/B: HIP hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4)
# x self-play lanes (slot groups on their own streams).  With 4 queues a
# third lane shares a queue with another stream (profiles/r2/hw_queues.txt).
# Usage (GPU box): bash profiles/r5/ab_queues.sh <tag> [connect_n|chess]
set -o pipefail
tag=${1:-q}
game=${2:-connect_n}
out=gpurun_out/$tag
mkdir -p "$out"
for q in 4 8; do
  for lanes in 2 3 4; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --game $game --no-cpu-baseline --lanes $lanes \
        > "$out/${game}_q${q}_l${lanes}.json" 2> "$out/${game}_q${q}_l${lanes}.err" || { tail -5 "$out/${game}_q${q}_l${lanes}.err"; exit 1; }
    python - "$out/${game}_q${q}_l${lanes}.json" "$q" "$lanes" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"queues {sys.argv[2]} lanes {sys.argv[3]}: {d['metric']} value {d['value']:.1f} ms/step {d['ms_per_step']:.2f} "
      f"exp/s {d.get('expansions_per_s', 0):.3g} frac {d['roofline']['frac']:.4f}", flush=True)
PY
  done
done
