"""oracle/az_cpu.c (bench.py's native CPU baseline): its fp32 forward
against the float64 Keras restatement, and its self-play loop runs on
several threads with the shared cache."""
import numpy as np

import cpu_native
import keras_ref
import oracle
from custom_alphazero.model.weights import init_weights, weight_spec


def test_native_forward_matches_keras_restatement():
    for (H, W, grav) in [(6, 7, True), (5, 5, False)]:
        A = W if grav else H * W
        w = init_weights(weight_spec(H, W, A, depth=2), seed=3, randomize_bn=True)
        flat = cpu_native.fold_for_cpu(w, H, W, A, depth=2)
        rng = np.random.RandomState(1)
        boards = rng.randint(-1, 2, (6, H, W)).astype(np.int8)
        rp, rv = keras_ref.forward(w, oracle.full_state(boards), depth=2)
        for i, b in enumerate(boards):
            p, v = cpu_native.forward(flat, b, grav, depth=2)
            assert np.abs(p - rp[i]).max() < 1e-5 and abs(v - rv[i]) < 1e-5


def test_native_selfplay_threads():
    w = init_weights(weight_spec(6, 7, 7, depth=1), seed=0)
    flat = cpu_native.fold_for_cpu(w, 6, 7, 7, depth=1)
    r = cpu_native.selfplay(flat, 6, 7, 4, True, 8, depth=1, threads=3, seconds=0.5)
    assert r["games"] >= 3 and r["plies"] >= 7 * r["games"]
    assert r["expansions"] == r["evaluations"] + r["cache_hits"]
