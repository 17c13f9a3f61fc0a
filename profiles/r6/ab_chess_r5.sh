#!/bin/bash
# chess configs[4] opening line: round 5's tree (profiles/ab_trees/r5, its own
# bench.py + libaz) against this tree, cache off and on (round 6)
set -o pipefail
mkdir -p gpurun_out/r6/ab_chess
R=$PWD
run() {  # name dir args...
  local n=$1 d=$2; shift 2
  (cd $d && timeout -k 10 300 python3 bench.py --game chess --no-cpu-baseline "$@") > gpurun_out/r6/ab_chess/$n.json 2> gpurun_out/r6/ab_chess/$n.err || { echo "FAIL $n"; tail -3 gpurun_out/r6/ab_chess/$n.err; return 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6/ab_chess/$n.json').read().strip().splitlines()[-1])
tc=d.get('transposition_cache') or {}
print('$n', d['value'], 'ms/step', d['ms_per_step'], 'tower us', round(d['roofline']['avg_launch_ms']*1e3,1), 'hit', tc.get('hit_rate'), flush=True)"
}
for i in 1 2; do
  run r5_$i $R/profiles/ab_trees/r5 || exit 1
  run r6c0_$i $R --cache-log2 0 || exit 1
  run r6c20_$i $R --cache-log2 20 || exit 1
done
