"""Isolated forward timing of the current libaz (AZ_LIB_PATH for A/B builds):
HIP-event time of the timed region per forward at the given batch sizes."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402
from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    algo = int(os.environ.get("AZ_ALGO", "0"))
    rng = np.random.RandomState(5)
    H, W = (int(v) for v in os.environ.get("AZ_HW", "6,7").split(","))  # 9,9: configs[2]'s board
    n = 4 if (H, W) == (6, 7) else 5
    spec = weight_spec(H, W, W, depth=4)
    w = init_weights(spec, seed=0, randomize_bn=True)
    out = []
    for nb in [int(v) for v in os.environ.get("AZ_BATCHES", "673,1346,4096").split(",")]:
        xx = oracle.full_state(rng.randint(-1, 2, (nb, H, W)).astype(np.int8))
        eng = az.Engine(H, W, n, True, 25, slots=max(nb, 2048), evaluator=az.EVAL_NETWORK, depth=4,
                        conv_algo=algo, tower_natural_order=os.environ.get("AZ_NATURAL") == "1")
        eng.set_weights(w.items())
        eng.forward(xx)
        eng.timer(True)
        for _ in range(20):
            eng.forward(xx)
        st = eng.stats()
        eng.timer(False)
        per = st["conv_ms"] / 20
        out.append(f"B={nb} {per * 1e3:.1f}us {nb * 313.8e6 * H * W / 42 / (per * 1e-3) / 1e12:.0f}TF")
        eng.close()
    print(tag, "algo", algo, " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
