#!/bin/bash
# chess: round 5's tree vs this tree with round 5's synchronous window and with the async drained window
set -o pipefail
mkdir -p gpurun_out/r6/ab_chess
R=$PWD
run() {
  local n=$1 d=$2; shift 2
  (cd $d && timeout -k 10 300 env "$@" python3 bench.py --game chess --no-cpu-baseline) > gpurun_out/r6/ab_chess/$n.json 2> gpurun_out/r6/ab_chess/$n.err || { echo "FAIL $n"; tail -3 gpurun_out/r6/ab_chess/$n.err; return 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6/ab_chess/$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], 'ms/step', d['ms_per_step'], 'tower us', round(d['roofline']['avg_launch_ms']*1e3,1), flush=True)"
}
for i in 1 2; do
  run r5w_$i $R/profiles/ab_trees/r5 X=1 || exit 1
  run r6sync_$i $R X=1 || exit 1
  run r6async_$i $R AZ_CHESS_ASYNC_WINDOW=1 || exit 1
done
