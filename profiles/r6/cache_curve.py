#!/usr/bin/env python3
"""Transposition-cache hit rate and ms/move against moves played (round 6).

configs[1] exactly as bench.py runs it (4096 C4 slots, S=100, the random-init
128f x 4 network, 8 HIP queues, bounded pooled arenas), one line per --every
moves: the window's hit rate (cache hits / expansions), ms per move, games/s
(games finished on the device / window time), the entries the table holds and
its generation.  Usage: cache_curve.py --cache-log2 25 --moves 900
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--cache-log2", type=int, default=25)
ap.add_argument("--moves", type=int, default=900)
ap.add_argument("--every", type=int, default=20)
ap.add_argument("--slots", type=int, default=4096)
ap.add_argument("--sims", type=int, default=100)
args = ap.parse_args()

from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402

spec = weight_spec(6, 7, 7, depth=4)
w = init_weights(spec, seed=0)
eng = az.Engine(6, 7, 4, True, args.sims, slots=args.slots, evaluator=az.EVAL_NETWORK, depth=4,
                cache_log2=args.cache_log2, compact=True, arena_edges=8 * args.sims * 7 + 42 * 7)
eng.set_weights(w.items())
eng.selfplay_begin(first_game=0, n_games=args.slots * (2 + args.moves // 7), base_seed=0)
prev = eng.stats()
t = time.perf_counter()
for m in range(1, args.moves + 1):
    eng.selfplay_step(1, sync=False)
    eng.selfplay_drain()
    if m % args.every == 0:
        st = eng.stats()
        now = time.perf_counter()
        d = {k: st[k] - prev[k] for k in ("expansions", "cache_hits", "games_done", "evaluations")}
        print(json.dumps({"cache_log2": args.cache_log2, "move": m,
                          "hit_rate": round(d["cache_hits"] / max(d["expansions"], 1), 4),
                          "ms_per_move": round(1e3 * (now - t) / args.every, 3),
                          "games_per_s": round(d["games_done"] / (now - t), 1),
                          "evals_per_move": d["evaluations"] // args.every,
                          "entries": st["cache_entries"], "capacity": st["cache_capacity"],
                          "fill": round(st["cache_entries"] / max(st["cache_capacity"], 1), 4),
                          "inserts_over_cap": round(st["cache_inserts"] / max(st["cache_capacity"], 1), 3),
                          "generation": st["cache_generation"], "errors": st["errors"]}), flush=True)
        assert st["errors"] == 0, st["errors"]
        prev, t = st, time.perf_counter()
