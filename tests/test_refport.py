"""The CPU-baseline port (oracle/refport.py) is the reference's algorithm:
pinned against the golden vectors the reference produced."""
import numpy as np
import pytest

import refport


@pytest.mark.parametrize("name,games", [("c4_s25", 4), ("c4_s100", 1), ("c5_9x9_s50", 1),
                                        ("nograv_5x5_s25", 2), ("c4_s1", 2)])
def test_refport_matches_reference(golden, name, games):
    z = golden("mcts_" + name)
    H, W, n, grav, S, A = (int(z[k]) for k in ("height", "width", "n", "gravity", "sims",
                                                "action_space"))
    off = 0
    for g in range(games):
        r = refport.play_game(H, W, n, bool(grav), S, int(z["seed"][g]), refport.SynthEval(A))
        T = int(z["game_len"][g])
        sl = slice(off, off + T)
        assert r["T"] == T
        np.testing.assert_array_equal(r["moves"], z["moves"][sl])
        np.testing.assert_array_equal(r["policies"].view(np.uint64), z["policy"][sl].view(np.uint64))
        np.testing.assert_array_equal(r["states"], z["state"][sl])
        np.testing.assert_array_equal(r["rewards"], z["reward"][sl])
        assert r["expansions"] == z["expansions"][g]
        off += T


def test_torch_cpu_net_matches_keras_restatement():
    import keras_ref
    from custom_alphazero.model.weights import init_weights, weight_spec
    w = init_weights(weight_spec(6, 7, 7), seed=3, randomize_bn=True)
    net = refport.TorchCPUNet(w, depth=4)
    b = refport.PortBoard(6, 7, 4, True)
    for a in (3, 3, 2, 4, 0):
        b.play(a)
    p, v = net(b)
    rp, rv = keras_ref.forward(w, b.state()[None], depth=4)
    assert np.abs(p - rp[0]).max() < 1e-5 and abs(v - rv[0]) < 1e-5
