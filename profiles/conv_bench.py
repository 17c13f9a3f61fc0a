#!/usr/bin/env python3
"""Forward-pass microbenchmark: az_forward on B random Connect-4 boards, the
conv kernels timed with the engine's HIP events (same method as bench.py).
Usage: python3 profiles/conv_bench.py [B] [reps] [algo: 0 one-launch tower, 1 fp32 direct, 2 fp16x2 per layer]
[H W] (default 6 7; the 9x9 Connect-5 board of configs[2]: 9 9)
TFLOP/s are direct-convolution (algorithmic) FLOP per second."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
import numpy as np  # noqa: E402

from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
H, W = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (6, 7)
algo = int(sys.argv[3]) if len(sys.argv) > 3 else az.CONV_F16X2
eng = az.Engine(H, W, 4 if (H, W) == (6, 7) else 5, True, 1, slots=B, evaluator=az.EVAL_NETWORK, conv_algo=algo)
eng.set_weights(init_weights(weight_spec(H, W, W), seed=0).items())
rng = np.random.RandomState(0)
b = rng.randint(-1, 2, (B, H, W)).astype(np.int8)
x = np.zeros((B, H, W, 4), np.float32)
x[..., 0], x[..., 1], x[..., 2], x[..., 3] = b == 0, b == 1, b == -1, 1
eng.forward(x)
eng.timer(True)
t0 = time.perf_counter()
for _ in range(reps):
    eng.forward(x)
wall = time.perf_counter() - t0
st = eng.stats()
flop = B * H * W * 2 * 128 * 128 * 19 * 4
avg = st["conv_ms"] / st["conv_launches"]  # (the tower: one launch per forward, else one per conv)
print(f"algo={algo} B={B} reps={reps}: conv {st['conv_ms'] / reps:.3f} ms/forward ({avg * 1e3:.1f} us/launch), "
      f"{flop * reps / (st['conv_ms'] * 1e-3) / 1e12:.1f} TFLOP/s; wall {wall / reps * 1e3:.2f} ms/forward incl. H2D/D2H")
