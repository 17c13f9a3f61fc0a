#!/bin/bash
# End-of-round rocprof collection on the final build, then the other BASELINE configs.
set -o pipefail
bash profiles/collect_r2.sh > gpurun_out/collect_r2.log 2>&1 || { tail -20 gpurun_out/collect_r2.log; exit 1; }
head -30 gpurun_out/prof_r2/summary.md
bash profiles/bench_configs.sh || exit 1
for f in s400 s400_32k c5_9x9; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['unit'], d['ms_per_step'], d['expansions_per_s'], d['roofline']['frac'], d['transposition_cache']['hit_rate'])" gpurun_out/configs/$f.json; done
