#!/bin/bash
# Alternating chess (configs[4] shard) bench lines of A/B libraries (round 6):
#   ab_chess.sh TAG name... [-- bench args]; "prod" = the in-tree libaz, else
#   profiles/ab_libs/<name>/libaz.so (AZ_LIB_PATH)
set -o pipefail
TAG=$1; shift
names=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p gpurun_out/r6/abc_$TAG
i=0
for n in "${names[@]}"; do
  i=$((i+1))
  if [ "$n" == "prod" ]; then unset AZ_LIB_PATH; else export AZ_LIB_PATH=$PWD/profiles/ab_libs/$n/libaz.so; fi
  out=gpurun_out/r6/abc_$TAG/${i}_$n.json
  timeout -k 10 300 python3 bench.py --game chess --no-cpu-baseline "$@" > $out 2> ${out%.json}.err || { echo "FAIL $n"; tail -5 ${out%.json}.err; exit 1; }
  python3 - "$out" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:10s} {d['value']:11.1f} {d['unit']}  ms/step {d['ms_per_step']:8.3f}  tower {r['avg_launch_ms']*1e3:6.1f} us  "
      f"build {r.get('build_id')}", flush=True)
PY
done
