#!/usr/bin/env python3
"""Chess forward microbenchmark: az_chess_forward on B random (8,8,118)
states (one-hot piece planes), the tower convs timed with the engine's HIP
events like bench.py.  Usage: python3 profiles/chess_conv_bench.py [B] [reps]
TFLOP/s are direct-convolution (algorithmic) FLOP of the 8 tower convs."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
import numpy as np  # noqa: E402

from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
eng = az.ChessEngine(1, slots=B, evaluator=az.EVAL_NETWORK)
eng.set_weights(init_weights(weight_spec(8, 8, 1880, in_channels=118), seed=0).items())
rng = np.random.RandomState(0)
x = np.zeros((B, 8, 8, 118), np.float32)
piece = rng.randint(0, 13, (B, 8, 8))
for h in (6, 7):
    x[..., h * 14:(h + 1) * 14][np.arange(B)[:, None, None], np.arange(8)[None, :, None],
                                np.arange(8)[None, None, :], piece] = 1.0
x[..., 112:116] = 1.0
x[..., 116] = 1.0
eng.forward(x)
eng.timer(True)
t0 = time.perf_counter()
for _ in range(reps):
    eng.forward(x)
wall = time.perf_counter() - t0
st = eng.stats()
flop = B * 64 * 2 * 128 * 128 * 19 * 4
avg = st["conv_ms"] / max(st["conv_launches"], 1)
print(f"chess B={B} reps={reps}: tower {st['conv_ms'] / reps:.3f} ms/forward ({avg * 1e3:.1f} us/launch), "
      f"{flop * reps / (st['conv_ms'] * 1e-3) / 1e12:.1f} TFLOP/s; wall {wall / reps * 1e3:.2f} ms/forward")
