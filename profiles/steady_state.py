"""Per-move trace of the bench workload (C4, S=100, 4096 slots): games
finished, cache hit rate and ms per move, from the first move on.  Used to
choose bench.py's untimed pre-roll (the window must not depend on --warmup).

python profiles/steady_state.py --moves 200 > gpurun_out/steady.jsonl
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--moves", type=int, default=200)
    ap.add_argument("--slots", type=int, default=4096)
    ap.add_argument("--sims", type=int, default=100)
    ap.add_argument("--cache-log2", type=int, default=25)
    args = ap.parse_args()
    import torch
    from custom_alphazero import engine as az
    from custom_alphazero.model.weights import init_weights, weight_spec
    spec = weight_spec(6, 7, 7)
    eng = az.Engine(6, 7, 4, True, args.sims, slots=args.slots, evaluator=az.EVAL_NETWORK,
                    cache_log2=args.cache_log2)
    eng.set_weights(init_weights(spec, seed=0).items())
    eng.selfplay_begin(0, args.slots * 64, 0)
    prev = eng.stats()
    for mv in range(args.moves):
        t0 = time.perf_counter()
        st = eng.selfplay_step(1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        d = {k: st[k] - prev[k] for k in ("games_done", "expansions", "cache_hits", "evaluations")}
        print(json.dumps({"move": mv, "ms": round(1e3 * dt, 2), "games": d["games_done"],
                          "hit_rate": round(d["cache_hits"] / max(d["expansions"], 1), 4),
                          "evals": d["evaluations"], "expansions": d["expansions"],
                          "gen": st["cache_generation"]}), flush=True)
        prev = st


if __name__ == "__main__":
    main()
