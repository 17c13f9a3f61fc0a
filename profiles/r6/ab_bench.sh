#!/bin/bash
# Alternating bench.py runs of A/B libraries (round 6): ab_bench.sh TAG name... [-- bench args]
# name "prod" = the in-tree libaz, else profiles/ab_libs/<name>/libaz.so (AZ_LIB_PATH)
set -o pipefail
TAG=$1; shift
names=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p gpurun_out/r6/ab_$TAG
i=0
for n in "${names[@]}"; do
  i=$((i+1))
  if [ "$n" == "prod" ]; then unset AZ_LIB_PATH; else export AZ_LIB_PATH=$PWD/profiles/ab_libs/$n/libaz.so; fi
  out=gpurun_out/r6/ab_$TAG/${i}_$n.json
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cache-window "$@" > $out 2> ${out%.json}.err || { echo "FAIL $n"; tail -5 ${out%.json}.err; exit 1; }
  python3 - "$out" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:10s} {d['value']:9.1f} games/s  ms/step {d['ms_per_step']:7.3f}  lanes {d['lanes']}  "
      f"hit {d['transposition_cache']['hit_rate'] if d['transposition_cache'] else None}  tower {r['avg_launch_ms']*1e3:6.1f} us "
      f"x {r.get('boards_per_launch')} boards  iso {r.get('isolated', {}).get('avg_launch_ms')}  "
      f"tree {d['roofline_tree']['avg_launch_ms']*1e3:.1f} us  build {r.get('build_id')}", flush=True)
PY
done
