#!/usr/bin/env python3
"""Max |GPU - float64 restatement| of the network outputs per conv algorithm
(argv[1]: 0 AZ_CONV_F16X2, 1 AZ_CONV_DIRECT): Connect-4 and chess, random
positions and weights with non-trivial BatchNorm statistics."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("custom-alphazero_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import numpy as np  # noqa: E402
ALGO = int(sys.argv[1]) if len(sys.argv) > 1 else 0

import keras_ref  # noqa: E402
from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402


def randomize_bn(w, seed):
    rng = np.random.default_rng(seed)
    for k in list(w):
        if k.endswith(".mean"):
            w[k] = rng.normal(0, 0.1, w[k].shape).astype(np.float32)
        elif k.endswith(".var"):
            w[k] = rng.uniform(0.5, 1.5, w[k].shape).astype(np.float32)
    return w


w = randomize_bn(init_weights(weight_spec(6, 7, 7), seed=1), 0)
eng = az.Engine(6, 7, 4, True, 1, slots=512, evaluator=az.EVAL_NETWORK, conv_algo=ALGO)
eng.set_weights(w.items())
rng = np.random.RandomState(0)
b = rng.randint(-1, 2, (512, 6, 7))
x = np.stack([b == 0, b == 1, b == -1, np.ones_like(b, bool)], -1).astype(np.float32)
p, v = eng.forward(x)
rp, rv = keras_ref.forward(w, x, depth=4)
print(f"conv_algo={ALGO} C4: max|dp| {np.abs(p - rp).max():.3e} "
      f"max|dv| {np.abs(v - rv).max():.3e}")
import chess_oracle as C  # noqa: E402
wc = randomize_bn(init_weights(weight_spec(8, 8, 1880, in_channels=118), seed=3), 1)
ce = az.ChessEngine(16, slots=128, evaluator=az.EVAL_NETWORK, conv_algo=ALGO)
ce.set_weights(wc.items())
pos, roots = C.random_positions(128, seed=5)
xs = np.stack([C.full_state(*C.reference_history(q, bool(r)), q) for q, r in zip(pos, roots)]).astype(np.float32)
p, v = ce.forward(xs)
rp, rv = keras_ref.forward(wc, xs, depth=4)
print(f"conv_algo={ALGO} chess: max|dp| {np.abs(p - rp).max():.3e} "
      f"max|dv| {np.abs(v - rv).max():.3e}")
