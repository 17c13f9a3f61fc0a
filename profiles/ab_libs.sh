#!/bin/bash
# in-bench A/B of libaz builds (AZ_LIB_PATH): bash profiles/ab_libs.sh <variant>...
set -o pipefail
mkdir -p gpurun_out/ab_libs
for spec in "$@"; do
  v=${spec%%:*}; flags=""; [ "$spec" != "$v" ] && flags="${spec#*:}"; flags=${flags//,/ }
  if [ "$v" = base ]; then lib=custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=profiles/ab_libs/$v/libaz.so; fi
  AZ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline $flags > gpurun_out/ab_libs/$spec.json 2> gpurun_out/ab_libs/$spec.err || { tail gpurun_out/ab_libs/$spec.err; exit 1; }
  python3 - "gpurun_out/ab_libs/$spec.json" "$spec" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], d["value"], d["ms_per_step"], "conv_ms", r["avg_launch_ms"], "iso", r["isolated"]["avg_launch_ms"], "union", r["busy_union"]["frac"], "busy_ms", r["conv_busy_ms"])
PY
done
