"""Host enqueue cost of a self-play move: bench.py's configuration (C4, 4096
slots, S=100, network, 2 lanes), time of selfplay_step(sync=False) calls
(the host enqueues 2 lanes x 100 simulations x ~12 launches) against the
GPU time per move.  Usage: python profiles/host_enqueue.py"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "custom-alphazero_amd"))
import torch  # noqa: E402
from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402

spec = weight_spec(6, 7, 7)
w = init_weights(spec, seed=0)
eng = az.Engine(6, 7, 4, True, 100, slots=4096, evaluator=az.EVAL_NETWORK, cache_log2=25, compact=True)
eng.set_weights([(n, w[n]) for n, _ in spec])
eng.selfplay_begin(0, 4096 * 20, 0)
for _ in range(30):
    eng.selfplay_step(1)
    eng.selfplay_drain()
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for _ in range(10):
    a = time.perf_counter()
    eng.selfplay_step(1, sync=False)
    host.append(time.perf_counter() - a)
    eng.selfplay_drain()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 10
print(f"host enqueue per move: mean {1e3 * sum(host) / len(host):.2f} ms (min {1e3 * min(host):.2f}, "
      f"max {1e3 * max(host):.2f}); wall per move {1e3 * wall:.2f} ms; "
      f"{1e6 * sum(host) / len(host) / (100 * 2 * 12):.1f} us per launch (approx.)")
