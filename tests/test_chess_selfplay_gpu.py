"""Chess self-play on the GPU (csrc/az_chess_mcts.hip, BASELINE configs[4])
against the chess oracle's MCTS (oracle/chess_oracle.c): the synthetic
evaluator pins the tree arithmetic bit for bit (moves, root positions,
MCTS.play policies, expansion counts, terminations); the network evaluator
is checked against the float64 Keras restatement (1e-5) and replayed through
the oracle with the engine's own batch-1 outputs."""
import numpy as np
import pytest

import chess_oracle as C

pytestmark = pytest.mark.gpu
NET_TOL = 1e-5


def _engine(**kw):
    from custom_alphazero import engine as az
    return az.ChessEngine(**kw)


def _compare(r, g, ref, tag):
    T = int(r["lengths"][g])
    assert T == ref["T"], (tag, g, T, ref["T"])
    assert r["terminations"][g] == ref["termination"], (tag, g)
    assert r["results"][g] == ref["result"], (tag, g)
    assert r["expansions"][g] == ref["expansions"], (tag, g)
    assert np.array_equal(r["moves"][g, :T], ref["moves"]), (tag, g)
    assert r["positions"][g, :T].tobytes() == ref["positions"].tobytes(), (tag, g)
    assert np.array_equal(r["policy_n"][g, :T], ref["policy_n"]), (tag, g)
    for t in range(T):
        n = ref["policy_n"][t]
        assert np.array_equal(r["policy_actions"][g, t, :n], ref["policy_actions"][t, :n]), (tag, g, t)
        assert np.array_equal(r["policy_probs"][g, t, :n].view(np.uint64),
                              ref["policy_probs"][t, :n].view(np.uint64)), (tag, g, t)


@pytest.mark.parametrize("sims,plies,slots,games,greedy,lanes,cache", [
    (24, 40, 3, 5, 8, 1, 0),      # slot refill, the reference's greedy threshold (never reached)
    (24, 40, 3, 5, 8, 3, 0),      # same games on three streams: results do not depend on lanes
    (16, 30, 4, 4, 1, 2, 0),      # greedy from the first move (one-hot policy, one draw consumed)
    (8, 400, 4, 6, 8, 2, 0),      # long games: checkmate / stalemate / 75-move / cap terminations
    (2, 60, 2, 2, 8, 1, 0),       # S=2: the root expansion plus one visit
    # round 6: the transposition cache + per-simulation dedup (identical games
    # at the start: every slot's leaves coincide), and a table small enough
    # to fill and evict (LRU) while other lanes read it
    (24, 40, 3, 5, 8, 1, 16), (24, 40, 6, 8, 8, 3, 16), (8, 400, 4, 6, 8, 2, 16), (32, 60, 8, 8, 8, 2, 6),
])
def test_chess_selfplay_synthetic_matches_oracle(sims, plies, slots, games, greedy, lanes, cache):
    from custom_alphazero import engine as az
    eng = _engine(mcts_iterations=sims, slots=slots, evaluator=az.EVAL_SYNTHETIC, max_plies=plies,
                  index_move_greedy=greedy, lanes=lanes, cache_log2=cache)
    st = eng.selfplay_run(0, games, 1000)
    r = eng.selfplay_results()
    assert st["errors"] == 0 and st["games_done"] == games
    if cache == 16:  # the cache served leaves (and dedup shared rows): fewer network rows than expansions
        assert st["cache_hits"] > 0 and st["evaluations"] + st["cache_hits"] < st["expansions"]
    if cache == 6:  # 64 entries: filled, then evicted many times over
        assert st["cache_generation"] >= 2 * 16 and st["cache_entries"] == 2 ** 6
    for g in range(games):
        ref = C.play_game(sims, 1000 + g, plies, greedy_ply=greedy)
        _compare(r, g, ref, "synthetic")
    eng.close()


def test_chess_synthetic_evaluator_matches_oracle():
    """The device synthetic evaluator = orc_chess_synth (indirectly: one
    expansion's priors are its normalised output)."""
    p, v = C.synth(C.from_fen(), 1)
    assert p.dtype == np.float32 and -1 <= v < 1 and ((p * 64) % 1 == 0).all()


@pytest.fixture(scope="module")
def chess_net():
    from custom_alphazero import engine as az
    from custom_alphazero.model.weights import init_weights, weight_spec
    spec = weight_spec(8, 8, 1880, in_channels=118)
    w = init_weights(spec, seed=3)
    # non-trivial BatchNorm statistics so the folding is exercised
    rng = np.random.default_rng(0)
    for k in list(w):
        if k.endswith(".mean"):
            w[k] = rng.normal(0, 0.1, w[k].shape).astype(np.float32)
        elif k.endswith(".var"):
            w[k] = rng.uniform(0.5, 1.5, w[k].shape).astype(np.float32)
    eng = _engine(mcts_iterations=16, slots=64, evaluator=az.EVAL_NETWORK, max_plies=12, lanes=2)
    eng.set_weights(w.items())
    yield eng, w
    eng.close()


def _states(n, seed):
    pos, roots = C.random_positions(n, seed=seed)
    x = np.stack([C.full_state(*C.reference_history(p, bool(r)), p) for p, r in zip(pos, roots)])
    return x.astype(np.float32)


@pytest.mark.parametrize("algo", ["f16x2", "direct", "f16x2_layers"])
def test_chess_forward_matches_keras_restatement(chess_net, algo):
    """Every algorithm -- the one-launch tower (AZ_CONV_F16X2: stem, tower and
    head 1x1 convs in one kernel), fp32 direct, the per-layer fp16x2 chain --
    against the float64 restatement, and batch invariant."""
    import keras_ref
    from custom_alphazero import engine as az
    eng, w = chess_net
    if algo != "f16x2":
        eng = _engine(mcts_iterations=16, slots=64, evaluator=az.EVAL_NETWORK, max_plies=12,
                      conv_algo=az.CONV_DIRECT if algo == "direct" else az.CONV_F16X2_LAYERS)
        eng.set_weights(w.items())
    x = _states(96, seed=21)  # more than one engine chunk (64 slots)
    probs, values = eng.forward(x)
    rp, rv = keras_ref.forward(w, x, depth=4)
    assert np.abs(probs - rp).max() < NET_TOL
    assert np.abs(values - rv).max() < NET_TOL
    # batch invariance (the replay parity below depends on it)
    p1, v1 = eng.forward(x[5:6])
    assert np.array_equal(p1[0], probs[5]) and v1[0] == values[5]
    if algo != "f16x2":
        eng.close()


def test_chess_tower_reports_its_launch():
    """The chess forward is one tower launch per simulation (plus the dense
    heads): the conv timer sees one launch per forward, and the engine
    reports the tower's issued MFMA FLOP per board."""
    from custom_alphazero import engine as az
    from custom_alphazero.model.weights import init_weights, weight_spec
    eng = _engine(mcts_iterations=8, slots=64, evaluator=az.EVAL_NETWORK, max_plies=4)
    eng.set_weights(init_weights(weight_spec(8, 8, 1880, in_channels=118), seed=1).items())
    eng.timer(True)
    eng.forward(_states(64, seed=2))
    st = eng.stats()
    eng.timer(False)
    assert st["conv_launches"] == 1 and st["issued_flop_per_board"] > 3 * 64 * 2 * 128 * 128 * 19 * 4 * 0.8
    eng.close()


def _chess_range_weights(S=2.0 ** 18):
    """The same function as seed-7 weights with the stem's and block 0 conv1's
    outputs S times larger (BN gamma/beta scaled; ReLU is positively
    homogeneous) and the next convs' kernels divided by S: activations far
    past the fp16 split range (|x| > 32752)."""
    from custom_alphazero.model.weights import init_weights, weight_spec
    w = init_weights(weight_spec(8, 8, 1880, depth=2, in_channels=118), seed=7, randomize_bn=True)
    for u in ("stem", "block0.conv1"):
        w[u + ".gamma"] = (w[u + ".gamma"] * S).astype(np.float32)
        w[u + ".beta"] = (w[u + ".beta"] * S).astype(np.float32)
    for u in ("block0.conv1", "block0.res", "block0.conv2"):
        w[u + ".kernel"] = (w[u + ".kernel"] / S).astype(np.float32)
    return w


def test_chess_activation_range_is_rescaled_not_failed():
    """activations past the fp16 split range.  The chess
    tower stores such a board's layer at a power-of-two scale: the forward
    stays within NET_TOL of the float64 restatement and self-play completes
    (the per-layer chain reports a device error instead)."""
    import keras_ref
    from custom_alphazero import engine as az
    w = _chess_range_weights()
    x = _states(40, seed=9)
    stem = keras_ref.inner(np.asarray(x, np.float64), w, "stem", 1e-3)
    assert stem.max() > 32752 * 4
    rp, rv = keras_ref.forward(w, x, depth=2)
    eng = _engine(mcts_iterations=8, slots=64, evaluator=az.EVAL_NETWORK, max_plies=6, depth=2)
    eng.set_weights(w.items())
    p, v = eng.forward(x)
    assert np.abs(p - rp).max() < NET_TOL and np.abs(v - rv).max() < NET_TOL
    st = eng.selfplay_run(0, 8, 5)
    assert st["errors"] == 0 and st["games_done"] == 8
    eng.close()
    lay = _engine(mcts_iterations=8, slots=64, evaluator=az.EVAL_NETWORK, max_plies=6, depth=2,
                  conv_algo=az.CONV_F16X2_LAYERS)
    lay.set_weights(w.items())
    with pytest.raises(az.AzError, match="activation-range"):
        lay.selfplay_run(0, 8, 5)
    lay.close()


@pytest.mark.parametrize("cache", [0, 18])
def test_chess_selfplay_network_replays_on_oracle(chess_net, cache):
    eng, w = chess_net
    if cache:  # the same network on an engine with the transposition cache
        from custom_alphazero import engine as az
        eng = _engine(mcts_iterations=16, slots=64, evaluator=az.EVAL_NETWORK, max_plies=12, lanes=2,
                      cache_log2=cache)
        eng.set_weights(w.items())
    st = eng.selfplay_run(0, 3, 77)
    r = eng.selfplay_results()
    if cache:  # the three games search identically until their first draw: dedup shares rows
        assert st["evaluations"] + st["cache_hits"] < st["expansions"]

    def cb(pos, initial):
        x = C.full_state(*C.reference_history(pos, bool(initial)), pos)[None].astype(np.float32)
        p, v = eng.forward(x)
        return p[0], float(v[0])

    for g in range(3):
        ref = C.play_game(16, 77 + g, 12, callback=cb)
        _compare(r, g, ref, "network")
    if cache:
        eng.close()


def test_chess_engine_errors():
    from custom_alphazero import engine as az
    with pytest.raises(az.AzError, match="az_chess_engine_set_weights"):
        eng = _engine(mcts_iterations=4, slots=2, evaluator=az.EVAL_NETWORK)
        eng.selfplay_begin(0, 1, 0)
    with pytest.raises(az.AzError, match="arena"):
        eng = _engine(mcts_iterations=64, slots=2, evaluator=az.EVAL_SYNTHETIC, arena_edges=300)
        eng.selfplay_run(0, 2, 0)


def test_chess_play_api_matches_oracle():
    """self_play.play with ConfigGeneral.game == "chess": states are the
    reference's Board.full_state of each parent board, policies the dense
    MCTS.play policy, rewards alternate from the final result."""
    from custom_alphazero import self_play
    from custom_alphazero.config import ConfigGeneral, ConfigSelfPlay
    from custom_alphazero.mcts.mcts import SyntheticEvaluator
    saved = (ConfigGeneral.game, ConfigSelfPlay.mcts_iterations, ConfigSelfPlay.chess_max_plies,
             ConfigSelfPlay.chess_concurrent_games)
    try:
        ConfigGeneral.game = "chess"
        ConfigSelfPlay.mcts_iterations, ConfigSelfPlay.chess_max_plies = 12, 24
        ConfigSelfPlay.chess_concurrent_games = 2
        states, policies, rewards, records = self_play.play("run", {}, model=SyntheticEvaluator(),
                                                            n_games=3, base_seed=500)
    finally:
        (ConfigGeneral.game, ConfigSelfPlay.mcts_iterations, ConfigSelfPlay.chess_max_plies,
         ConfigSelfPlay.chess_concurrent_games) = saved
    off = 0
    for g in range(3):
        ref = C.play_game(12, 500 + g, 24)
        T = ref["T"]
        assert records[g].length == T and np.array_equal(records[g].moves, ref["moves"])
        for t in range(T):
            x = C.full_state(*C.reference_history(ref["positions"][t], t == 0), ref["positions"][t])
            assert np.array_equal(states[off + t].astype(np.float64), x), (g, t)
            dense = np.zeros(1880)
            n = ref["policy_n"][t]
            dense[ref["policy_actions"][t, :n]] = ref["policy_probs"][t, :n]
            assert np.array_equal(policies[off + t], dense), (g, t)
        exp = np.repeat(ref["result"], T)
        exp[-2::-2] = -exp[-2::-2]
        assert np.array_equal(rewards[off:off + T], exp)
        off += T
    assert off == len(states) == len(policies) == len(rewards)


@pytest.mark.parametrize("lanes", [1, 2])
def test_chess_drain_returns_every_game_once(lanes):
    """az_chess_selfplay_drain (ABI 10): asynchronous steps, a drain after
    each -- the games of the newest move whose snapshot is complete, never
    waiting for the running one -- then the rest after a synchronize: every
    game once, each record equal to az_chess_selfplay_results' rows."""
    import torch
    from custom_alphazero import engine as az
    eng = az.ChessEngine(mcts_iterations=10, slots=6, evaluator=az.EVAL_SYNTHETIC, max_plies=9, lanes=lanes)
    n_games = 20
    eng.selfplay_begin(300, n_games, 4)
    parts = []
    for _ in range(60):  # more moves than the batch needs (9-ply cap, 6 slots); idle slots skip
        eng.selfplay_step(1, sync=False)
        parts.append(eng.selfplay_drain())
    torch.cuda.synchronize()
    st = eng.stats()  # synchronizes the lanes
    assert st["active_slots"] == 0 and st["errors"] == 0
    parts.append(eng.selfplay_drain())
    assert len(eng.selfplay_drain()["lengths"]) == 0
    got = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    assert sorted(got["game_ids"].tolist()) == list(range(300, 300 + n_games))
    ref = eng.selfplay_results()
    gi = got["game_ids"] - 300
    for k in ("lengths", "results", "terminations", "expansions", "moves", "policy_n", "policy_actions"):
        np.testing.assert_array_equal(got[k], ref[k][gi], err_msg=k)
    np.testing.assert_array_equal(got["positions"].view(np.uint8), ref["positions"][gi].view(np.uint8))
    np.testing.assert_array_equal(got["policy_probs"].view(np.uint64), ref["policy_probs"][gi].view(np.uint64))
    # and the games are the oracle's
    for i in range(3):
        r = C.play_game(10, 4 + 300 + i, 9)
        g = int(np.nonzero(got["game_ids"] == 300 + i)[0][0])
        assert got["lengths"][g] == r["T"]
        np.testing.assert_array_equal(got["moves"][g, :r["T"]], r["moves"])
    eng.close()
