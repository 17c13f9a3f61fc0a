#!/bin/bash
# Bucketed transposition cache (16-slot buckets, cap/16 per generation, 6 live; the in-tree
# build) vs the linear-probe table with the same generations (lin16l6) and the bucketed table
# with round 2's cap/8, 2 live (b8l2).  GPU suite on the in-tree build first; then in-bench
# A/B and a 400-move per-move trace of base and b8l2 (stationarity).
set -o pipefail
mkdir -p gpurun_out/steady gpurun_out/r2t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r2t/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2t/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2t/gpu_tests.log
bash profiles/ab_libs.sh base lin16l6 b8l2 base lin16l6 b8l2 || exit 1
for v in base b8l2; do
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
