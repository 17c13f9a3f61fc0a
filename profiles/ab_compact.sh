set -o pipefail
mkdir -p gpurun_out/abc
for c in 1 0 1 0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-cache-window --compact $c >> gpurun_out/abc/c4.jsonl 2>> gpurun_out/abc/err.txt || exit 1
done
timeout -k 10 300 python bench.py --game chess --no-cpu-baseline > gpurun_out/abc/chess.json 2>> gpurun_out/abc/err.txt || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/abc/c4.jsonl"):
    d = json.loads(l)
    print(d["tree_arena"]["compact"], d["value"], d["ms_per_step"], d["tree_arena"]["max_retained_edges"], d["tree_arena"]["bytes_total"])
d = json.loads(open("gpurun_out/abc/chess.json").read().strip().splitlines()[-1])
print("chess", d["value"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"])
PY
