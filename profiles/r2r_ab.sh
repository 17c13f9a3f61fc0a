#!/bin/bash
# GPU suite with hit-refresh in the transposition cache, then in-bench A/B
# against the previous build (old = no refresh), warmup 5 and 60 (stationarity).
set -o pipefail
out=gpurun_out/r2r
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
bash profiles/ab_libs.sh old base old base old:--warmup,60 base:--warmup,60
for f in gpurun_out/ab_libs/*.json; do python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['transposition_cache']
print(sys.argv[1], d['value'], c['hit_rate'], c['generation_at_window_end'], c['age_moves_at_window_start'], c['live_entries'], d['untimed_moves'])" $f; done
