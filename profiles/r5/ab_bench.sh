#!/bin/bash
# in-bench A/B of libaz variants (AZ_LIB_PATH), alternating, games/s and the
# tower roofline fields: bash profiles/r4/ab_bench.sh <rounds> "<bench args>" base v1 ...
# (a variant "name:VAR=value" is the product library run with that environment setting)
set -o pipefail
rounds=$1; args=$2; shift 2
mkdir -p gpurun_out
for r in $(seq $rounds); do
  for v in "$@"; do
    envs=""
    if [ "${v#*:}" != "$v" ]; then envs=${v#*:}; v=${v%%:*}; lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so
    elif [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
    env $envs AZ_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > gpurun_out/abb_$v.json 2> gpurun_out/abb_$v.err || exit 1
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/abb_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],1), 'frac', r['frac'], 'union', r.get('busy_union',{}).get('frac'), 'launch_ms', r.get('avg_launch_ms'), 'boards', r.get('boards_per_launch'), flush=True)"
  done
done
