#!/bin/bash
# The timed window's HIP events (tower launch timer) on vs off, same library,
# alternating (round 6): ab_events.sh TAG [pairs]
set -o pipefail
TAG=$1; N=${2:-2}
mkdir -p gpurun_out/r6/abe_$TAG
for i in $(seq 1 $N); do
  for ev in 1 0; do
    out=gpurun_out/r6/abe_$TAG/${i}_ev$ev.json
    AZ_BENCH_WINDOW_EVENTS=$ev timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window > $out 2> ${out%.json}.err \
      || { echo "FAIL ev$ev"; tail -5 ${out%.json}.err; exit 1; }
    python3 - "$out" "events=$ev" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:10s} {d['value']:9.1f} games/s  ms/step {d['ms_per_step']:7.3f}  build {d['roofline'].get('build_id')}", flush=True)
PY
  done
done
