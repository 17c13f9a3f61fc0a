#!/bin/bash
# Cache generation layout A/B (all with hit-refresh): base = cap/8 per generation,
# 2 live; g16l6 = cap/16, 6 live; g8l3 = cap/8, 3 live.  In-bench games/s (preroll
# until generation 8) and a 400-move per-move trace of each (stationarity).
set -o pipefail
mkdir -p gpurun_out/steady
bash profiles/ab_libs.sh base g16l6 g8l3 base g16l6 g8l3 || exit 1
for v in base g16l6 g8l3; do
  if [ $v = base ]; then lib=custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=profiles/ab_libs/$v/libaz.so; fi
  AZ_LIB_PATH=$PWD/$lib timeout -k 10 200 python profiles/steady_state.py --moves 400 > gpurun_out/steady/$v.jsonl 2> gpurun_out/steady/$v.err || exit 1
  python3 - gpurun_out/steady/$v.jsonl $v <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for a in range(0, 400, 50):
    w = rows[a:a + 50]
    h = sum(r["hit_rate"] * r["expansions"] for r in w) / sum(r["expansions"] for r in w)
    print(sys.argv[2], f"moves {a}-{a+49}: hit {h:.4f} ms/move {sum(r['ms'] for r in w)/len(w):.2f} gen {w[-1]['gen']}")
PY
done
