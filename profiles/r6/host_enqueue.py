#!/usr/bin/env python3
"""Is the configs[1] step host-bound?  (round 6)  bench.py's setup (2^26 LRU
cache preroll to stationarity, 3 lanes, 8 HIP queues), then per move the host
time of selfplay_step(sync=False) (the enqueue of 100 simulations x lanes x 3
launches) and of the drain, against the move's wall time; with and without
the HIP-event timer bench.py runs in its window."""
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402
import torch  # noqa: E402

spec = weight_spec(6, 7, 7, depth=4)
eng = az.Engine(6, 7, 4, True, 100, slots=4096, evaluator=az.EVAL_NETWORK, depth=4,
                cache_log2=int(os.environ.get("CACHE_LOG2", "26")), compact=True, arena_edges=8 * 100 * 7 + 42 * 7)
eng.set_weights(init_weights(spec, seed=0).items())
eng.selfplay_begin(first_game=0, n_games=4096 * 700, base_seed=0)
moves = 0
while True:
    st = eng.selfplay_step(1)
    eng.selfplay_drain()
    moves += 1
    if moves >= 24 and st["cache_inserts"] >= 1.5 * st["cache_capacity"]:
        break
print(json.dumps({"preroll_moves": moves}), flush=True)
for timer in (False, True):
    eng.timer(timer)
    torch.cuda.synchronize()
    enq, dr = [], []
    t0 = time.perf_counter()
    for _ in range(30):
        a = time.perf_counter()
        eng.selfplay_step(1, sync=False)
        b = time.perf_counter()
        eng.selfplay_drain()
        c = time.perf_counter()
        enq.append(b - a)
        dr.append(c - b)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 30
    eng.timer(False)
    print(json.dumps({"timer": timer, "ms_per_move": round(1e3 * wall, 3),
                      "enqueue_ms_mean": round(1e3 * sum(enq) / 30, 3), "enqueue_ms_max": round(1e3 * max(enq), 3),
                      "drain_ms_mean": round(1e3 * sum(dr) / 30, 3), "lanes": eng.lanes}), flush=True)
