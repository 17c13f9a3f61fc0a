"""AZ_EVAL_HOST: the reference's duck-typed evaluator seam (mcts/mcts.py:130-137,
``self.model(np.expand_dims(board.full_state, 0))``) on the device search.

A plain Python callable stands in for the model.  With the synthetic
evaluator written as such a callable (oracle/synth.py over the full_state
planes the engine hands it), the search must reproduce the reference's own
golden games bit for bit -- the same fixtures the compiled-in synthetic
evaluator is pinned to; with the network's az_forward as the callable, it must
reproduce the device network evaluator's games exactly."""
import numpy as np
import pytest

import synth
from custom_alphazero import engine as az
from custom_alphazero import self_play
from custom_alphazero.config import ConfigConnectN, ConfigSelfPlay
from custom_alphazero.connect_n.board import Board
from custom_alphazero.model.weights import init_weights, weight_spec
from test_engine_gpu import check_selfplay_game, selfplay_games

pytestmark = pytest.mark.gpu


class SynthModel:
    """model(x) -> (probabilities [n, A], value [n, 1]) like the reference's
    PolicyValueModel call, computing oracle/synth.py's evaluator; records the
    batch sizes it was called with."""

    def __init__(self, action_space):
        self.A = action_space
        self.calls = []

    def __call__(self, x):
        self.calls.append(len(x))
        p = np.zeros((len(x), self.A), np.float32)
        v = np.zeros((len(x), 1), np.float32)
        for i, st in enumerate(x):
            own, opp = synth.masks_from_full_state(st)
            probs, value = synth.synth_eval(own, opp, self.A)
            p[i] = probs
            v[i] = value
        return p, v


def host_engine(z, slots, model, cache_log2=0, lanes=0, compact=False):
    H, W, n, grav, S = (int(z[k]) for k in ("height", "width", "n", "gravity", "sims"))
    eng = az.Engine(H, W, n, bool(grav), S, slots=slots, evaluator=az.EVAL_HOST,
                    cache_log2=cache_log2, lanes=lanes, compact=compact)
    eng.set_host_evaluator(model)
    return eng


@pytest.mark.parametrize("name,cache_log2,lanes", [("c4_s25", 0, 1), ("c4_s25", 16, 2),
                                                   ("nograv_5x5_s25", 16, 1), ("c5_9x9_s50", 0, 2)])
def test_selfplay_host_callable_matches_reference(golden, name, cache_log2, lanes):
    """Batched self-play with the evaluator a Python callable: every game equal
    to the reference's play_game (moves, f64 policies, states, rewards,
    expansions), with and without the cache, on one or two lanes."""
    z = golden("mcts_" + name)
    seeds = z["seed"].astype(np.int64)
    model = SynthModel(int(z["action_space"]))
    eng = host_engine(z, len(seeds), model, cache_log2, lanes, compact=True)
    games = selfplay_games(eng, int(seeds[0]), len(seeds))
    for g, got in enumerate(games):
        check_selfplay_game(z, g, got)
    # batched: one call per simulation and lane, never more leaves than slots
    assert max(model.calls) <= len(seeds) and len(model.calls) < sum(int(g["expansions"]) for g in games)
    eng.close()


@pytest.fixture
def game_cfg():
    saved = (ConfigConnectN.board_height, ConfigConnectN.board_width, ConfigConnectN.n,
             ConfigConnectN.gravity, ConfigSelfPlay.mcts_iterations)

    def set_(z):
        ConfigConnectN.board_height, ConfigConnectN.board_width = int(z["height"]), int(z["width"])
        ConfigConnectN.n, ConfigConnectN.gravity = int(z["n"]), bool(z["gravity"])
        ConfigSelfPlay.mcts_iterations = int(z["sims"])

    yield set_
    (ConfigConnectN.board_height, ConfigConnectN.board_width, ConfigConnectN.n,
     ConfigConnectN.gravity, ConfigSelfPlay.mcts_iterations) = saved


def test_play_game_with_any_callable_model_matches_reference(golden, game_cfg, monkeypatch):
    """self_play.play_game(model=<a callable>) -> MCTS(model=...) as the reference
    builds it: the games equal the reference's own, the tree views carry its
    edge statistics."""
    z = golden("mcts_c4_s25")
    game_cfg(z)
    model = SynthModel(int(z["action_space"]))
    off = 0
    for g, seed in enumerate(z["seed"][:2]):
        monkeypatch.setattr(self_play.time, "time", lambda s=seed: float(s))
        states, policies, rewards, mcts = self_play.play_game(
            0, Board.get_all_possible_moves(), int(z["sims"]), "test-run", {}, model=model)
        T = int(z["game_len"][g])
        sl = slice(off, off + T)
        np.testing.assert_array_equal(states, z["state"][sl])
        np.testing.assert_array_equal(policies.view(np.uint64), z["policy"][sl].view(np.uint64))
        np.testing.assert_array_equal(rewards, z["reward"][sl])
        node = mcts.root
        for ply in range(T):
            k = int(z["n_edges"][off + ply])
            assert [e.visit_count for e in node.edges] == z["edge_n"][off + ply, :k].tolist()
            node = [e for e in node.edges if e.played][0].child
        off += T
        monkeypatch.undo()
    assert max(model.calls) == 1  # one tree: batch-1 calls, as the reference makes them


def test_host_callable_network_equals_device_network():
    """The network's own forward as the host callable == the device network
    evaluator: identical games (the forward is batch invariant)."""
    H, W, S, G = 6, 7, 16, 24
    w = init_weights(weight_spec(H, W, W, depth=4), seed=3, randomize_bn=True)
    net = az.Engine(H, W, 4, True, S, slots=G, evaluator=az.EVAL_NETWORK, depth=4, cache_log2=16)
    net.set_weights(w.items())
    fwd = az.Engine(H, W, 4, True, S, slots=G, evaluator=az.EVAL_NETWORK, depth=4)
    fwd.set_weights(w.items())
    host = az.Engine(H, W, 4, True, S, slots=G, evaluator=az.EVAL_HOST, depth=4, cache_log2=16)
    host.set_host_evaluator(lambda x: fwd.forward(x))
    a = selfplay_games(net, 0, G, base_seed=11)
    b = selfplay_games(host, 0, G, base_seed=11)
    for ga, gb in zip(a, b):
        assert ga["T"] == gb["T"]
        np.testing.assert_array_equal(ga["moves"], gb["moves"])
        np.testing.assert_array_equal(ga["policy"].view(np.uint64), gb["policy"].view(np.uint64))
        assert ga["expansions"] == gb["expansions"]
    for e in (net, fwd, host):
        e.close()


def test_host_evaluator_errors():
    """No callable -> AZ_E_STATE; an exception inside the callable ends the
    search and is re-raised; a wrong output shape is an error too."""
    eng = az.Engine(6, 7, 4, True, 8, slots=1, evaluator=az.EVAL_HOST)
    eng.tree_reset([0], np.zeros((1, 6, 7), np.int8))
    with pytest.raises(az.AzError, match="set_evaluator"):
        eng.tree_search(4)

    def boom(x):
        raise ValueError("model failed")

    eng.set_host_evaluator(boom)
    eng.tree_reset([0], np.zeros((1, 6, 7), np.int8))
    with pytest.raises(ValueError, match="model failed"):
        eng.tree_search(4)
    eng.set_host_evaluator(lambda x: (np.zeros((len(x), 3), np.float32), np.zeros(len(x), np.float32)))
    eng.tree_reset([0], np.zeros((1, 6, 7), np.int8))
    with pytest.raises(ValueError):
        eng.tree_search(4)
    good = SynthModel(7)
    eng.set_host_evaluator(good)
    eng.tree_reset([0], np.zeros((1, 6, 7), np.int8))
    eng.tree_search(4)
    assert good.calls
    eng.close()
    with pytest.raises(az.AzError):  # only an AZ_EVAL_HOST engine takes a callable
        e2 = az.Engine(6, 7, 4, True, 8, slots=1, evaluator=az.EVAL_SYNTHETIC)
        try:
            e2.set_host_evaluator(good)
        finally:
            e2.close()
