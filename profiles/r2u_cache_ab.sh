#!/bin/bash
# Live window of the bucketed cache: base (2^25, cap/16 per generation, 6 live), l10 (10 live),
# base on 2^26 / 2^27 tables.  In-bench games/s, then per-move traces of l10 and 2^27.
set -o pipefail
mkdir -p gpurun_out/steady
bash profiles/ab_libs.sh base l10 base:--cache-log2,26 base:--cache-log2,27 base l10 base:--cache-log2,27 || exit 1
trace() {  # variant lib moves log2
  AZ_LIB_PATH=$PWD/$2 timeout -k 10 300 python profiles/steady_state.py --moves $3 --cache-log2 $4 > gpurun_out/steady/$1.jsonl 2> gpurun_out/steady/$1.err || exit 1
  python3 - gpurun_out/steady/$1.jsonl $1 $3 <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for a in range(0, int(sys.argv[3]), 100):
    w = rows[a:a + 100]
    h = sum(r["hit_rate"] * r["expansions"] for r in w) / sum(r["expansions"] for r in w)
    print(sys.argv[2], f"moves {a}-{a+99}: hit {h:.4f} ms/move {sum(r['ms'] for r in w)/len(w):.2f} gen {w[-1]['gen']}")
PY
}
trace l10 profiles/ab_libs/l10/libaz.so 600 25
trace c27 custom-alphazero_amd/custom_alphazero/_lib/libaz.so 1000 27
