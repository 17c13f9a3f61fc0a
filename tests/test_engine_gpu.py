"""GPU parity of libaz against the reference (golden vectors) and the oracle.

Bar: bit-exact visit counts, W, priors, policies and
moves; network outputs within 1e-5 of the float64 Keras restatement.
"""
import numpy as np
import pytest

import keras_ref
import oracle
from custom_alphazero import engine as az
from custom_alphazero.model.weights import init_weights, weight_spec
from test_oracle import MCTS_FIXTURES, NOISE_FIXTURES, check_game_against_golden

pytestmark = pytest.mark.gpu

NET_TOL = 1e-5  # north_star: value/policy outputs within 1e-5 (fp32)


def synth_engine(z, slots, cache_log2=0, lanes=0, compact=False):
    H, W, n, grav, S = (int(z[k]) for k in ("height", "width", "n", "gravity", "sims"))
    noise = bool(z["dirichlet_noise"])
    kw = dict(dirichlet_noise=True, dirichlet_alpha=float(z["dirichlet_alpha"]),
              dirichlet_ratio=float(z["dirichlet_ratio"])) if noise else {}
    return az.Engine(H, W, n, bool(grav), S, slots=slots, evaluator=az.EVAL_SYNTHETIC,
                     cache_log2=cache_log2, lanes=lanes, compact=compact, **kw)


def selfplay_games(eng, first, n_games, base_seed=0):
    eng.selfplay_run(first, n_games, base_seed)
    r = eng.selfplay_results()
    games = []
    for g in range(n_games):
        T = int(r["lengths"][g])
        res = int(r["results"][g])
        rewards = np.full(T, res, np.int64)
        rewards[-2::-2] *= -1
        games.append(dict(T=T, moves=r["moves"][g, :T], policy=r["policies"][g, :T],
                          boards=r["boards"][g, :T], rewards=rewards,
                          expansions=int(r["expansions"][g])))
    return games


def check_selfplay_game(z, g, got):
    lens = z["game_len"]
    off = int(lens[:g].sum())
    T = int(lens[g])
    sl = slice(off, off + T)
    assert got["T"] == T, (g, got["T"], T)
    np.testing.assert_array_equal(got["moves"], z["moves"][sl])
    np.testing.assert_array_equal(got["policy"].view(np.uint64), z["policy"][sl].view(np.uint64))
    np.testing.assert_array_equal(oracle.full_state(got["boards"]), z["state"][sl])
    np.testing.assert_array_equal(got["rewards"], z["reward"][sl])
    assert got["expansions"] == z["expansions"][g]


@pytest.mark.parametrize("cache_log2,lanes,compact", [(0, 1, False), (16, 1, False), (16, 2, False),
                                                      (0, 1, True), (16, 2, True)])
@pytest.mark.parametrize("name", MCTS_FIXTURES)
def test_selfplay_synthetic_matches_reference(golden, name, cache_log2, lanes, compact):
    """Batched device self-play == the reference's play_game, game by game,
    with and without the shared transposition cache (plays_inferences), on one
    stream or two lanes (slot groups on separate streams sharing the cache),
    and with the left subtrees reclaimed after every move (compact)."""
    z = golden("mcts_" + name)
    seeds = z["seed"].astype(np.int64)
    assert np.all(np.diff(seeds) == 1)
    for slots in sorted({len(seeds), max(1, len(seeds) // 2)}):  # also exercises slot refill
        eng = synth_engine(z, slots, cache_log2, lanes, compact)
        games = selfplay_games(eng, int(seeds[0]), len(seeds))
        for g, got in enumerate(games):
            check_selfplay_game(z, g, got)
        eng.close()


@pytest.mark.parametrize("cache_log2,lanes,compact", [(0, 1, False), (16, 2, True)])
@pytest.mark.parametrize("name", NOISE_FIXTURES)
def test_selfplay_dirichlet_noise_matches_reference(golden, name, cache_log2, lanes, compact):
    """SURVEY 8 a8 / VERDICT r3 item 9: with ConfigMCTS.enable_dirichlet_noise
    every root selection mixes np.random.dirichlet(0.03 * ones(k)) from the
    game's stream into the priors (mcts.py:70-85).  Device self-play (the
    select kernels draw the legacy gamma variates on each game's MT19937)
    == the reference's play_game with noise on: moves, policies, states,
    rewards and expansion counts bitwise, on the reference's own fixtures."""
    z = golden("mcts_" + name)
    seeds = z["seed"].astype(np.int64)
    assert np.all(np.diff(seeds) == 1) and bool(z["dirichlet_noise"])
    for slots in sorted({len(seeds), max(1, len(seeds) // 2)}):
        eng = synth_engine(z, slots, cache_log2, lanes, compact)
        games = selfplay_games(eng, int(seeds[0]), len(seeds))
        for g, got in enumerate(games):
            check_selfplay_game(z, g, got)
        eng.close()


@pytest.mark.parametrize("shape", [(6, 7, 4, True, 50), (5, 5, 4, False, 20)])
def test_selfplay_dirichlet_noise_many_games_vs_oracle(shape):
    """128 noisy games (every simulation draws a Dirichlet vector at the root)
    on 48 slots == the C oracle, whose draws call libm log / pow exactly as
    numpy does, game by game and bitwise.  The device's log / pow restate
    glibc 2.35's (csrc/az_random.h, az_libm_tables.h), so every draw equals
    the host's bit for bit (tests/test_dirichlet_cpu.py: 0 mismatches over
    10^6 arguments of each kind)."""
    H, W, n, grav, S = shape
    eng = az.Engine(H, W, n, grav, S, slots=48, evaluator=az.EVAL_SYNTHETIC, dirichlet_noise=True,
                    lanes=2, compact=True, cache_log2=16)
    games = selfplay_games(eng, 0, 128, base_seed=777)
    eng.close()
    for g, got in enumerate(games):
        ref = oracle.play_game(H, W, n, grav, S, 777 + g, noise=(0.03, 0.25))
        assert got["T"] == ref["T"], g
        np.testing.assert_array_equal(got["moves"], ref["moves"])
        np.testing.assert_array_equal(got["policy"].view(np.uint64), ref["policy"].view(np.uint64))
        assert got["expansions"] == ref["expansions"], g


def test_selfplay_dirichlet_noise_network_replays_on_oracle():
    """Noise with the real network: the oracle, fed the engine's own batch-1
    network outputs and drawing the same root noise, reproduces every move
    and policy bit for bit."""
    eng, _ = make_net_engine(S=50, slots=16, dirichlet_noise=True, compact=True, cache_log2=16)
    games = selfplay_games(eng, 0, 16, base_seed=91)
    cache = {}

    def cb(board):
        k = board.tobytes()
        if k not in cache:
            p, v = eng.forward(oracle.full_state(board[None]))
            cache[k] = (p[0], float(v[0]))
        return cache[k]

    for g in (0, 7, 15):
        ref = oracle.play_game(6, 7, 4, True, 50, 91 + g, evaluator="callback", callback=cb, noise=(0.03, 0.25))
        assert games[g]["T"] == ref["T"]
        np.testing.assert_array_equal(games[g]["moves"], ref["moves"])
        np.testing.assert_array_equal(games[g]["policy"].view(np.uint64), ref["policy"].view(np.uint64))
    eng.close()


def test_tree_api_noise_needs_the_callers_draws():
    """A noisy engine's tree search takes the caller's np.random.dirichlet
    rows (az_tree_search_noise): a plain search is refused, too few rows
    fail loudly, the device never draws for the tree API."""
    eng = az.Engine(6, 7, 4, True, 10, slots=1, evaluator=az.EVAL_SYNTHETIC, dirichlet_noise=True)
    eng.tree_reset([0], np.zeros((1, 6, 7), np.int8))
    with pytest.raises(az.AzError, match="az_tree_search_noise"):
        eng.tree_search(5)
    with pytest.raises(az.AzError, match="root-noise-rows-exhausted"):
        eng.tree_search(5, noise=np.full((1, 3, 7), 1 / 7))  # an unexpanded root makes 4 selections
    eng.close()
    plain = az.Engine(6, 7, 4, True, 10, slots=1, evaluator=az.EVAL_SYNTHETIC)
    plain.tree_reset([0], np.zeros((1, 6, 7), np.int8))
    with pytest.raises(az.AzError, match="dirichlet_noise = 1"):
        plain.tree_search(5, noise=np.full((1, 5, 7), 1 / 7))
    plain.close()


@pytest.mark.parametrize("name", ["c4_s25", "c4_s100", "c5_9x9_s50", "nograv_5x5_s25", "c4_s1"] + NOISE_FIXTURES)
def test_tree_api_edges_match_reference(golden, name):
    """MCTS.search/play through the tree API: root edge N, W, prior bit-exact.
    Noisy fixtures: every root selection's np.random.dirichlet vector is drawn
    here from the game's stream, before play's draw, as the reference's
    select does (mcts.py:70-85, 111-120), and passed to the search."""
    z = golden("mcts_" + name)
    H, W, S = int(z["height"]), int(z["width"]), int(z["sims"])
    A = int(z["action_space"])
    noisy = bool(z["dirichlet_noise"])
    off = 0
    for g, seed in enumerate(z["seed"][:3]):
        eng = synth_engine(z, 1)
        eng.tree_reset([0], np.zeros((1, H, W), np.int8))
        rng = np.random.RandomState(int(seed))
        rng.rand(1, H, W, 4)  # play_game's model construction (model.py:167-169)
        T = int(z["game_len"][g])
        for ply in range(T):
            if noisy:
                before = eng.tree_export(0)
                rows = S if before["root_n"] > 0 else S - 1
                k = int(z["n_edges"][off + ply])
                noise = np.zeros((1, max(rows, 1), A))
                for r in range(rows):
                    noise[0, r, :k] = rng.dirichlet(np.ones(k) * float(z["dirichlet_alpha"]))
                eng.tree_search(S, noise=noise)
            else:
                eng.tree_search(S)
            t = eng.tree_export(0)
            k, f = t["root_n"], t["root_first"]
            gi = off + ply
            assert k == z["n_edges"][gi]
            np.testing.assert_array_equal(t["action"][f:f + k], z["edge_action"][gi, :k])
            np.testing.assert_array_equal(t["n"][f:f + k], z["edge_n"][gi, :k])
            np.testing.assert_array_equal(t["w"][f:f + k].view(np.uint64), z["edge_w"][gi, :k].view(np.uint64))
            np.testing.assert_array_equal(t["prior"][f:f + k].view(np.uint64),
                                          z["edge_prior"][gi, :k].view(np.uint64))
            moves, status, policy = eng.tree_play([rng.random_sample()], greedy=ply >= 8)
            assert moves[0] == z["moves"][gi]
            np.testing.assert_array_equal(policy[0].view(np.uint64), z["policy"][gi].view(np.uint64))
            assert (status[0] != 0) == (ply == T - 1)
        off += T
        eng.close()
    assert A == z["policy"].shape[1]


@pytest.mark.parametrize("cache_log2,lanes,compact", [(0, 1, False), (10, 1, False), (20, 1, False),
                                                      (20, 3, False), (0, 2, False), (20, 2, True)])
def test_selfplay_synthetic_many_games_vs_oracle(cache_log2, lanes, compact):
    """256 games at S=50 on 96 slots (heavy refill) == the C oracle, bitwise;
    cache_log2=10 fills the table (full buckets: the no-insert path); 2-3 lanes
    race on the shared cache and the refill counter; compact reclaims the
    left subtrees after every move."""
    eng = az.Engine(6, 7, 4, True, 50, slots=96, evaluator=az.EVAL_SYNTHETIC,
                    cache_log2=cache_log2, lanes=lanes, compact=compact)
    games = selfplay_games(eng, 1000, 256, base_seed=7)
    for g, got in enumerate(games):
        ref = oracle.play_game(6, 7, 4, True, 50, 7 + 1000 + g)
        assert got["T"] == ref["T"]
        np.testing.assert_array_equal(got["moves"], ref["moves"])
        np.testing.assert_array_equal(got["policy"].view(np.uint64), ref["policy"].view(np.uint64))
        np.testing.assert_array_equal(got["boards"], ref["boards"])
        assert got["expansions"] == ref["expansions"]
    st = eng.stats()
    assert st["games_done"] == 256 and st["errors"] == 0 and st["active_slots"] == 0
    if cache_log2:
        assert st["cache_hits"] > 0
        assert st["cache_hits"] + st["evaluations"] <= st["expansions"] + 0  # dedup only removes
    else:
        assert st["evaluations"] == st["expansions"] and st["cache_hits"] == 0


@pytest.mark.parametrize("lanes", [1, 2, 3])
def test_cache_eviction_generations_are_transparent(lanes):
    """A cache small enough to fill and turn over many times (az_tree.h: every
    entry is looked up, a hit moves it into the current generation, an insert
    into a full bucket evicts its least recently used entry 2+ generations old
    while other lanes read the table) leaves every game bitwise equal to the
    oracle."""
    eng = az.Engine(6, 7, 4, True, 50, slots=32, evaluator=az.EVAL_SYNTHETIC, cache_log2=17, lanes=lanes)
    games = selfplay_games(eng, 3000, 512, base_seed=9)
    st = eng.stats()
    assert st["cache_gen_size"] == 2 ** 17 // 16  # kCacheGenDiv
    assert st["cache_generation"] >= 24, st["cache_generation"]  # > 1.5 turnovers of the table
    assert st["cache_entries"] >= 0.99 * 2 ** 17, st["cache_entries"]  # full: inserts evicted entries
    assert st["cache_entries"] <= 2 ** 17
    assert st["cache_hits"] > 0 and st["errors"] == 0
    for g, got in enumerate(games):
        ref = oracle.play_game(6, 7, 4, True, 50, 9 + 3000 + g)
        assert got["T"] == ref["T"]
        np.testing.assert_array_equal(got["moves"], ref["moves"])
        np.testing.assert_array_equal(got["policy"].view(np.uint64), ref["policy"].view(np.uint64))
        assert got["expansions"] == ref["expansions"]
    # a generation must outlast three moves of every slot's inserts (the
    # lane-drift bound): cap/16 below it takes 3 * slots * sims + 1 inserts per
    # generation while that is at most cap/4; smaller tables only fill
    mid = az.Engine(6, 7, 4, True, 50, slots=32, evaluator=az.EVAL_SYNTHETIC, cache_log2=16, lanes=lanes)
    assert mid.stats()["cache_gen_size"] == 3 * 32 * 50 + 1
    small = az.Engine(6, 7, 4, True, 50, slots=32, evaluator=az.EVAL_SYNTHETIC, cache_log2=14, lanes=lanes)
    assert small.stats()["cache_gen_size"] == 0


@pytest.mark.parametrize("lanes", [1, 2])
def test_drain_returns_every_game_once(lanes):
    """az_selfplay_drain after each move hands every finished game to the host
    exactly once, with the same records az_selfplay_results returns."""
    eng = az.Engine(6, 7, 4, True, 20, slots=40, evaluator=az.EVAL_SYNTHETIC, cache_log2=12, lanes=lanes)
    n_games = 150
    eng.selfplay_begin(500, n_games, 3)
    parts, steps = [], 0
    while True:
        st = eng.selfplay_step(1)
        parts.append(eng.selfplay_drain(max_games=64 if steps % 2 else None))
        steps += 1
        if st["active_slots"] == 0:
            break
    while True:  # a capped drain may leave games behind
        d = eng.selfplay_drain()
        if not len(d["lengths"]):
            break
        parts.append(d)
    got = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    assert sorted(got["game_ids"].tolist()) == list(range(500, 500 + n_games))
    assert eng.stats()["games_drained"] == n_games
    ref = eng.selfplay_results()
    order = np.argsort(got["game_ids"])
    gi = got["game_ids"][order] - 500
    for k in ("lengths", "results", "expansions", "moves", "boards"):
        np.testing.assert_array_equal(got[k][order], ref[k][gi], err_msg=k)
    np.testing.assert_array_equal(got["policies"][order].view(np.uint64), ref["policies"][gi].view(np.uint64))
    assert len(eng.selfplay_drain()["lengths"]) == 0


@pytest.mark.parametrize("lanes", [1, 2])
def test_async_steps_drain_every_game_once(lanes):
    """selfplay_step(sync=False) returns without waiting; each drain returns the
    games of the newest move whose count snapshot is complete (never waiting
    for the running move), and after a synchronize the rest: every game once,
    records identical to az_selfplay_results, and the same games as a
    synchronous run of the batch."""
    import torch
    def run(sync):
        eng = az.Engine(6, 7, 4, True, 20, slots=40, evaluator=az.EVAL_SYNTHETIC, cache_log2=12, lanes=lanes,
                        compact=True)
        eng.selfplay_begin(100, 150, 5)
        parts = []
        for _ in range(200):  # more moves than any game needs; idle slots just skip
            eng.selfplay_step(1, sync=sync)
            parts.append(eng.selfplay_drain())
        torch.cuda.synchronize()
        parts.append(eng.selfplay_drain())
        parts.append(eng.selfplay_drain())  # nothing left
        assert len(parts[-1]["lengths"]) == 0
        return eng, {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    eng_a, got = run(False)
    assert sorted(got["game_ids"].tolist()) == list(range(100, 250))
    ref = eng_a.selfplay_results()
    order = np.argsort(got["game_ids"])
    gi = got["game_ids"][order] - 100
    for k in ("lengths", "results", "expansions", "moves", "boards"):
        np.testing.assert_array_equal(got[k][order], ref[k][gi], err_msg=k)
    np.testing.assert_array_equal(got["policies"][order].view(np.uint64), ref["policies"][gi].view(np.uint64))
    _, got_s = run(True)
    order_s = np.argsort(got_s["game_ids"])
    for k in ("lengths", "results", "expansions", "moves", "boards"):
        np.testing.assert_array_equal(got[k][order], got_s[k][order_s], err_msg=k)


def test_pow_table_is_python_pow(golden):
    z = golden("numerics")
    eng = az.Engine(6, 7, 4, True, 100, slots=1, evaluator=az.EVAL_SYNTHETIC,
                    max_tree_visits=2_000_001)
    tab = eng.pow_table(2_000_001)
    exc = z["pow_exceptions"]
    np.testing.assert_array_equal(tab[exc].view(np.uint64), z["pow_values"].view(np.uint64))
    mask = np.ones(len(tab), bool)
    mask[exc] = False
    np.testing.assert_array_equal(tab[mask], np.sqrt(np.arange(len(tab), dtype=np.float64))[mask])


@pytest.mark.parametrize("name", ["c4", "c5_9x9", "nograv_5x5"])
def test_encode_and_mask_match_reference(golden, name):
    z = golden("board_" + name)
    H, W, grav = int(z["height"]), int(z["width"]), bool(z["gravity"])
    eng = az.Engine(H, W, int(z["n"]), grav, 4, slots=512, evaluator=az.EVAL_SYNTHETIC)
    state, mask = eng.encode(z["array"])
    np.testing.assert_array_equal(state, oracle.full_state(z["array"]))
    np.testing.assert_array_equal(mask, z["mask"])


# ------------------------------------------------------------------ network
CONV_ALGOS = [az.CONV_F16X2, az.CONV_DIRECT, az.CONV_F16X2_LAYERS]


def make_net_engine(H=6, W=7, n=4, grav=True, S=25, slots=256, seed=0, randomize_bn=True, depth=4,
                    cache_log2=0, conv_algo=az.CONV_F16X2, lanes=0, compact=False, hidden=256, **kw):
    A = W if grav else W * H
    spec = weight_spec(H, W, A, depth=depth, hidden=hidden)
    w = init_weights(spec, seed=seed, randomize_bn=randomize_bn)
    eng = az.Engine(H, W, n, grav, S, slots=slots, evaluator=az.EVAL_NETWORK, depth=depth,
                    value_hidden=hidden, cache_log2=cache_log2, conv_algo=conv_algo, lanes=lanes,
                    compact=compact, **kw)
    eng.set_weights(w.items())
    return eng, w


def random_boards(rng, k, H, W):
    b = rng.randint(-1, 2, (k, H, W)).astype(np.int8)
    return b


@pytest.mark.parametrize("conv_algo", CONV_ALGOS)
@pytest.mark.parametrize("shape", [(6, 7, True), (9, 9, True), (5, 5, False), (7, 6, True)])
def test_forward_matches_keras_restatement(shape, conv_algo):
    """Every conv algorithm (the one-launch fp16x2 tower, fp32 direct, the
    per-layer fp16x2 kernels) within NET_TOL of the float64 Keras restatement;
    9x9 runs the tower's 192-row in-place tiles, 5x5 five boards per tile."""
    H, W, grav = shape
    eng, w = make_net_engine(H, W, 4, grav, slots=300, conv_algo=conv_algo)
    rng = np.random.RandomState(5)
    x = oracle.full_state(random_boards(rng, 37, H, W))
    x[-5:] = rng.rand(5, H, W, 4).astype(np.float32)  # arbitrary (non one-hot) inputs too
    p, v = eng.forward(x)
    rp, rv = keras_ref.forward(w, x, depth=4)
    assert np.abs(p - rp).max() < NET_TOL, np.abs(p - rp).max()
    assert np.abs(v - rv).max() < NET_TOL, np.abs(v - rv).max()
    np.testing.assert_allclose(p.sum(axis=1), 1.0, atol=1e-6)


@pytest.mark.parametrize("depth,hidden", [(0, 256), (1, 256), (17, 64), (2, 300)])
def test_forward_outside_the_tower_falls_back(depth, hidden):
    """the default conv_algo accepts any depth and value head
    size.  Networks the one-launch tower does not hold (depth 0 -- its heads
    run inside the last block --, depth > 16, value_hidden > 256) run the
    per-layer kernels instead, within NET_TOL of the float64 restatement."""
    eng, w = make_net_engine(6, 7, 4, True, slots=64, depth=depth, hidden=hidden)
    rng = np.random.RandomState(3)
    x = oracle.full_state(random_boards(rng, 20, 6, 7))
    p, v = eng.forward(x)
    rp, rv = keras_ref.forward(w, x, depth=depth)
    assert np.abs(p - rp).max() < NET_TOL, np.abs(p - rp).max()
    assert np.abs(v - rv).max() < NET_TOL, np.abs(v - rv).max()
    eng.selfplay_run(0, 2, 1)
    assert eng.stats()["errors"] == 0
    eng.close()


@pytest.mark.parametrize("shape", [(6, 7, True), (5, 5, False), (7, 6, True), (4, 5, True), (9, 9, True)])
def test_tower_slot_plan_is_bitwise_the_natural_order(shape):
    """The slot plan (border blocks skip the taps past their board edge: exact
    zeros not added) gives the same bits as the natural slot order
    (az_config.tower_natural_order), full and partial tiles, one-hot and
    arbitrary inputs."""
    H, W, grav = shape
    rng = np.random.RandomState(21)
    x = oracle.full_state(random_boards(rng, 37, H, W))
    x[-4:] = rng.rand(4, H, W, 4).astype(np.float32)
    out = []
    for natural in (False, True):
        eng, _ = make_net_engine(H, W, 4, grav, slots=300, conv_algo=az.CONV_F16X2,
                                 tower_natural_order=natural)
        out.append(eng.forward(x))
        out.append(eng.forward(x[:1]))
        eng.close()
    for a, b in zip(out[:2], out[2:]):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


def _range_weights(S=2.0 ** 18):
    """Weights whose stem output and block-0 conv1 output are S times the
    network's (BN gamma/beta scaled: ReLU is positively homogeneous) while the
    next convs' kernels are divided by S: the same function, with activations
    far beyond the fp16 split range (|x| > 32752)."""
    spec = weight_spec(6, 7, 7, depth=2)
    w = init_weights(spec, seed=4, randomize_bn=True)
    for u in ("stem", "block0.conv1"):
        w[u + ".gamma"] = (w[u + ".gamma"] * S).astype(np.float32)
        w[u + ".beta"] = (w[u + ".beta"] * S).astype(np.float32)
    for u in ("block0.conv1", "block0.res", "block0.conv2"):
        w[u + ".kernel"] = (w[u + ".kernel"] / S).astype(np.float32)
    # block0.conv1 saw an S-times input with a 1/S kernel, then its BN x S: its
    # output is S times; conv2's 1/S kernel brings block 0's sum back
    return w


def test_activation_range_is_rescaled_not_failed():
    """SURVEY 8 a18 + VERDICT r2 item 3: activations past the fp16 split range.
    The one-launch tower stores such a board's layer at a power-of-two scale
    and completes within NET_TOL of the float64 restatement, in self-play too;
    the per-layer path reports it as a device error instead of a wrong result."""
    w = _range_weights()
    rng = np.random.RandomState(9)
    x = oracle.full_state(random_boards(rng, 40, 6, 7))
    rp, rv = keras_ref.forward(w, x, depth=2)
    # the stem's activations really are out of the fp16 range
    stem = keras_ref.inner(np.asarray(x, np.float64), w, "stem", 1e-3)
    assert stem.max() > 32752 * 4
    eng = az.Engine(6, 7, 4, True, 16, slots=64, evaluator=az.EVAL_NETWORK, depth=2, conv_algo=az.CONV_F16X2)
    eng.set_weights(w.items())
    p, v = eng.forward(x)
    assert np.abs(p - rp).max() < NET_TOL and np.abs(v - rv).max() < NET_TOL
    eng.selfplay_run(0, 4, 3)
    assert eng.stats()["errors"] == 0
    eng.close()
    lay = az.Engine(6, 7, 4, True, 16, slots=64, evaluator=az.EVAL_NETWORK, depth=2,
                    conv_algo=az.CONV_F16X2_LAYERS)
    lay.set_weights(w.items())
    with pytest.raises(az.AzError, match="activation-range"):
        lay.selfplay_run(0, 4, 3)
    lay.close()


@pytest.mark.parametrize("conv_algo", CONV_ALGOS)
def test_forward_is_batch_invariant(conv_algo):
    eng, _ = make_net_engine(slots=512, conv_algo=conv_algo)
    rng = np.random.RandomState(11)
    x = oracle.full_state(random_boards(rng, 700, 6, 7))  # > slots: chunked
    p_all, v_all = eng.forward(x)
    for lo, hi in [(0, 1), (3, 4), (2, 5), (100, 229), (511, 513), (699, 700)]:
        p, v = eng.forward(x[lo:hi])
        np.testing.assert_array_equal(p, p_all[lo:hi])
        np.testing.assert_array_equal(v, v_all[lo:hi])


def test_tower_dual_launch_tiles_are_bitwise_equal():
    """Connect-4's dual tower launch (round 6, tower16_dual_kernel) runs
    96-row tiles of two boards when a launch holds at most 2 * CUs / lanes
    boards and 128-row tiles of three above: a board's outputs are the same
    bits either way (and within NET_TOL of the float64 restatement)."""
    eng, w = make_net_engine(slots=1024, conv_algo=az.CONV_F16X2, lanes=1)  # one lane: 96-row up to 512
    rng = np.random.RandomState(5)
    x = oracle.full_state(random_boards(rng, 900, 6, 7))
    p_big, v_big = eng.forward(x)            # 900 boards: 128-row tiles
    p_small, v_small = eng.forward(x[:301])  # 301 boards: 96-row tiles (one half-full)
    np.testing.assert_array_equal(p_small, p_big[:301])
    np.testing.assert_array_equal(v_small, v_big[:301])
    rp, rv = keras_ref.forward(w, x[:301], depth=4)
    assert np.abs(p_small - rp).max() < NET_TOL and np.abs(v_small - rv).max() < NET_TOL


@pytest.mark.parametrize("cache_log2,lanes", [(0, 1), (18, 1), (18, 2)])
def test_selfplay_network_replays_on_oracle(cache_log2, lanes):
    """Device self-play with the real network: the oracle, fed the engine's
    own batch-1 network outputs for every board it asks about, reproduces every
    move and visit-count policy bit for bit (replay parity)."""
    eng, _ = make_net_engine(S=40, slots=16, randomize_bn=False, cache_log2=cache_log2, lanes=lanes)
    games = selfplay_games(eng, 0, 6, base_seed=123)
    cache = {}

    def cb(board):
        key = board.tobytes()
        if key not in cache:
            p, v = eng.forward(oracle.full_state(board[None]))
            cache[key] = (p[0], float(v[0]))
        return cache[key]

    for g, got in enumerate(games):
        ref = oracle.play_game(6, 7, 4, True, 40, 123 + g, evaluator="callback", callback=cb)
        assert got["T"] == ref["T"]
        np.testing.assert_array_equal(got["moves"], ref["moves"])
        np.testing.assert_array_equal(got["policy"].view(np.uint64), ref["policy"].view(np.uint64))
        assert got["expansions"] == ref["expansions"]


@pytest.mark.parametrize("cfg", [(9, 9, 5, False, 30), (11, 11, 5, True, 30), (8, 8, 4, True, 40),
                                 (4, 4, 3, False, 20)])
@pytest.mark.parametrize("cache_log2", [0, 16])
def test_selfplay_synthetic_board_shapes_vs_oracle(cfg, cache_log2):
    """Shapes beyond the fixtures: A = 81 (serial select / wide expand and play
    kernels), the largest 11x11 board (121 of 128 cells), 8x8; slot refill."""
    H, W, n, grav, S = cfg
    games = 4
    for slots in (games, 2):
        eng = az.Engine(H, W, n, grav, S, slots=slots, evaluator=az.EVAL_SYNTHETIC,
                        cache_log2=cache_log2)
        got = selfplay_games(eng, 0, games, base_seed=31)
        for g in range(games):
            ref = oracle.play_game(H, W, n, grav, S, 31 + g)
            assert got[g]["T"] == ref["T"]
            np.testing.assert_array_equal(got[g]["moves"], ref["moves"])
            np.testing.assert_array_equal(got[g]["policy"].view(np.uint64), ref["policy"].view(np.uint64))
            np.testing.assert_array_equal(got[g]["boards"], ref["boards"])
            assert got[g]["expansions"] == ref["expansions"]
        eng.close()


def test_abi_error_behaviour():
    """Invalid arguments and states come back as AzError with a message (the
    ABI returns a negative code + az_last_error); nothing aborts."""
    with pytest.raises(az.AzError, match="n <= min"):
        az.Engine(6, 7, 7, True, 10, slots=4, evaluator=az.EVAL_SYNTHETIC)
    with pytest.raises(az.AzError, match="conv_algo"):
        az.Engine(6, 7, 4, True, 10, slots=4, evaluator=az.EVAL_NETWORK, conv_algo=5)
    with pytest.raises(az.AzError, match="lanes"):
        az.Engine(6, 7, 4, True, 10, slots=4, evaluator=az.EVAL_SYNTHETIC, lanes=-1)
    eng = az.Engine(6, 7, 4, True, 10, slots=4, evaluator=az.EVAL_NETWORK)
    with pytest.raises(az.AzError, match="set_weights"):
        eng.forward(np.zeros((1, 6, 7, 4), np.float32))
    with pytest.raises(az.AzError, match="set_weights"):
        eng.selfplay_run(0, 2, 0)
    eng.close()
    # a tree arena too small for the search is reported, not overrun
    eng = az.Engine(6, 7, 4, True, 50, slots=2, evaluator=az.EVAL_SYNTHETIC, arena_edges=64)
    with pytest.raises(az.AzError, match="arena-overflow"):
        eng.selfplay_run(0, 2, 0)
    eng.close()
    # play before any search
    eng = az.Engine(6, 7, 4, True, 10, slots=1, evaluator=az.EVAL_SYNTHETIC)
    eng.tree_reset([0], np.zeros((1, 6, 7), np.int8))
    with pytest.raises(az.AzError, match="play-before-search"):
        eng.tree_play([0.5])
    # ... which leaves the engine usable
    eng.tree_search(10)
    moves, status, _ = eng.tree_play([0.5])
    assert 0 <= moves[0] < 7 and status[0] == 0
    eng.close()


def test_compaction_bounds_the_arena_and_reports_overflow():
    """With compact, the slots of a lane share a pooled arena of two halves:
    a slot holds one move's search plus its kept subtree (a few thousand
    edges here, against S*H*W*A + A = 29.4k for a whole game at S=100); the
    retained and pool high-water marks are reported and stay inside; a pool
    too small for a search is a device error, not a wrong tree; results equal
    the uncompacted engine's bit for bit."""
    eng = az.Engine(6, 7, 4, True, 100, slots=64, evaluator=az.EVAL_SYNTHETIC, compact=True)
    eng.selfplay_run(0, 128, 3)
    st = eng.stats()
    assert st["errors"] == 0 and st["games_done"] == 128
    assert 0 < st["max_retained"] <= 8 * 100 * 7 + 42 * 7
    assert st["arena_pool_edges"] == 2 * 64 * st["arena_edges"]
    assert 0 < st["arena_pool_high"] <= 64 * (st["max_retained"] + 100 * 7 + 16 * 7)
    r = eng.selfplay_results()
    eng.close()
    ref = az.Engine(6, 7, 4, True, 100, slots=64, evaluator=az.EVAL_SYNTHETIC)
    ref.selfplay_run(0, 128, 3)
    rr = ref.selfplay_results()
    ref.close()
    for k in ("lengths", "moves", "expansions"):
        np.testing.assert_array_equal(r[k], rr[k])
    np.testing.assert_array_equal(r["policies"].view(np.uint64), rr["policies"].view(np.uint64))
    small = az.Engine(6, 7, 4, True, 100, slots=8, evaluator=az.EVAL_SYNTHETIC, compact=True, arena_edges=300)
    with pytest.raises(az.AzError, match="arena-overflow"):
        small.selfplay_run(0, 8, 3)
    small.close()


def _peaked(x):
    """A host evaluator that puts 90% of the prior on one action picked by a
    hash of the board, value 0: PUCT spends ~90% of a node's simulations
    below that child at every level, so the played (greedy) move keeps ~90%
    of the search and the kept subtree grows move after move (VERDICT r3
    item 2).  (A prior of ~1 instead makes the search a chain that stops
    at the first terminal position: small trees.)"""
    n, A = len(x), x.shape[2]
    cells = np.arange(1, x.shape[1] * x.shape[2] + 1)
    own = x[..., 1].reshape(n, -1) @ cells
    opp = x[..., 2].reshape(n, -1) @ cells
    a = (3 * own + 7 * opp).astype(np.int64) % A
    p = np.full((n, A), 0.1 / (A - 1), np.float32)
    p[np.arange(n), a] = 0.9
    return p, np.zeros(n, np.float32)


@pytest.mark.timeout(300)
def test_pooled_arena_holds_a_peaked_network():
    """A peaked evaluator over full games keeps large subtrees: some slots
    hold more than the per-slot average the pool was sized with (4000
    edges per half here: round 3's per-slot halves of that size would have
    overflowed, kErrArena), while the slots together fit -- the pooled halves
    are shared.  Every game equals the uncompacted engine's bit for bit."""
    S, slots, per_slot = 200, 32, 4000
    out = []
    for compact in (True, False):
        eng = az.Engine(6, 7, 4, True, S, slots=slots, evaluator=az.EVAL_HOST, compact=compact,
                        arena_edges=per_slot if compact else 0)
        eng.set_host_evaluator(_peaked)
        st = eng.selfplay_run(0, slots, 17)
        assert st["errors"] == 0 and st["games_done"] == slots
        out.append((eng.selfplay_results(), eng.stats()))
        eng.close()
    (r, st), (rr, _) = out
    assert st["arena_pool_edges"] == 2 * slots * per_slot
    assert st["max_retained"] > per_slot, st["max_retained"]  # one slot past the per-slot share
    assert st["arena_pool_high"] <= slots * per_slot
    for k in ("lengths", "moves", "expansions", "results"):
        np.testing.assert_array_equal(r[k], rr[k])
    np.testing.assert_array_equal(r["policies"].view(np.uint64), rr["policies"].view(np.uint64))
