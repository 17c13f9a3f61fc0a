#!/bin/bash
# GPU suite + default bench + a long-warmup bench (steady-state check).
# Usage (GPU box): bash profiles/gpu_check.sh <tag>
set -o pipefail
tag=${1:-r2}
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || { tail -30 "$out/gpu_tests.log"; exit 1; }
tail -3 "$out/gpu_tests.log"
timeout -k 10 300 python bench.py > "$out/bench_w5.json" 2> "$out/bench_w5.err" || { cat "$out/bench_w5.err"; exit 1; }
timeout -k 10 300 python bench.py --warmup 60 --no-cpu-baseline > "$out/bench_w60.json" 2> "$out/bench_w60.err" \
    || { cat "$out/bench_w60.err"; exit 1; }
python - "$out" <<'EOF'
import json, sys
for f in ("bench_w5.json", "bench_w60.json"):
    d = json.loads(open(f"{sys.argv[1]}/{f}").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["transposition_cache"]["hit_rate"], d["roofline"]["frac"])
EOF
