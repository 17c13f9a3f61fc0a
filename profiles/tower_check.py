"""Dev check of the one-launch tower (az_tower16.hip) against the per-layer
kernels and the float64 Keras restatement, plus isolated forward timings at
the bench's live batch (HIP events through az_timer_enable)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import keras_ref  # noqa: E402
import oracle  # noqa: E402
from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402


def make(H, W, grav, algo, slots, seed=0, scale=None):
    A = W if grav else W * H
    spec = weight_spec(H, W, A, depth=4)
    w = init_weights(spec, seed=seed, randomize_bn=True)
    if scale:
        for k in list(w):
            if k.endswith(".kernel") and (k.startswith("stem") or "block" in k):
                w[k] = (w[k] * scale).astype(np.float32)
    eng = az.Engine(H, W, 4, grav, 25, slots=slots, evaluator=az.EVAL_NETWORK, depth=4, conv_algo=algo)
    eng.set_weights(w.items())
    return eng, w


def main():
    rng = np.random.RandomState(5)
    for (H, W, grav) in [(6, 7, True), (9, 9, True), (5, 5, False)]:
        b = rng.randint(-1, 2, (37, H, W)).astype(np.int8)
        x = oracle.full_state(b)
        outs = {}
        for algo in (0, 1, 2):
            eng, w = make(H, W, grav, algo, 300)
            p, v = eng.forward(x)
            outs[algo] = (p, v)
            eng.close()
        rp, rv = keras_ref.forward(w, x, depth=4)
        for algo, (p, v) in outs.items():
            print(f"{H}x{W} algo {algo}: |dp| {np.abs(p - rp).max():.3g} |dv| {np.abs(v - rv).max():.3g}", flush=True)
    # activation range: weights x 40 push activations far past 32752
    b = rng.randint(-1, 2, (37, 6, 7)).astype(np.int8)
    x = oracle.full_state(b)
    eng, w = make(6, 7, True, 0, 300, scale=40.0)
    p, v = eng.forward(x)
    rp, rv = keras_ref.forward(w, x, depth=4)
    act = keras_ref.max_activation(w, x, depth=4) if hasattr(keras_ref, "max_activation") else None
    print(f"scaled x40 tower: |dp| {np.abs(p - rp).max():.3g} |dv| {np.abs(v - rv).max():.3g} maxact {act}",
          flush=True)
    eng.close()
    # batch invariance, tower
    eng, _ = make(6, 7, True, 0, 512)
    xx = oracle.full_state(rng.randint(-1, 2, (700, 6, 7)).astype(np.int8))
    pa, va = eng.forward(xx)
    ok = True
    for lo, hi in [(0, 1), (3, 4), (2, 5), (100, 229), (511, 513), (699, 700)]:
        p, v = eng.forward(xx[lo:hi])
        ok &= np.array_equal(p, pa[lo:hi]) and np.array_equal(v, va[lo:hi])
    print("batch invariant:", ok, flush=True)
    eng.close()
    # timings at the live batch
    for nb in (673, 1346, 4096):
        xx = oracle.full_state(rng.randint(-1, 2, (nb, 6, 7)).astype(np.int8))
        for algo in (0, 2):
            eng, _ = make(6, 7, True, algo, 2048 if nb <= 2048 else 4096)
            eng.forward(xx)
            eng.timer(True)
            for _ in range(20):
                eng.forward(xx)
            st = eng.stats()
            eng.timer(False)
            per_fwd = st["conv_ms"] / 20
            print(f"B={nb} algo {algo}: timed region per forward {per_fwd * 1e3:.1f} us "
                  f"({st['conv_launches']} launches), issued TF/s {nb * 313.8e6 / (per_fwd * 1e-3) / 1e12:.1f}",
                  flush=True)
            eng.close()


if __name__ == "__main__":
    main()
