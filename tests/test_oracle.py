"""Pin the CPU oracle against the reference's own outputs (golden vectors).

The golden vectors were produced by running the reference itself
(tests/golden/make_golden.py, numpy 1.26 legacy promotion).  These tests run
on CPU (no GPU marker): if the oracle drifts from the reference, every GPU
parity test that uses it as the checker is void.
"""
import math

import numpy as np
import pytest

import oracle
import synth

MCTS_FIXTURES = ["c4_s1", "c4_s2", "c4_s25", "c4_s100", "c4_s200", "c4_s400",
                 "c5_9x9_s50", "nograv_5x5_s25"]


def test_normalize_f32_matches_reference(golden):
    z = golden("numerics")
    for vin, vout, n, is64 in zip(z["norm_in"], z["norm_out"], z["norm_len"], z["norm_out_is64"]):
        out, uniform = oracle.normalize_f32(vin[:n])
        assert uniform == bool(is64)
        np.testing.assert_array_equal(out.view(np.uint64), vout[:n].view(np.uint64))


def test_normalize_visit_counts_matches_reference(golden):
    z = golden("numerics")
    for vin, vout, n in zip(z["visit_in"], z["visit_out"], z["visit_len"]):
        out = oracle.normalize_f64(vin[:n])
        np.testing.assert_array_equal(out.view(np.uint64), vout[:n].view(np.uint64))


def test_pow_half_is_libm_pow_not_sqrt(golden):
    z = golden("numerics")
    exc, val = z["pow_exceptions"], z["pow_values"]
    assert exc[0] == 2921 and len(exc) > 1000
    for k, v in zip(exc, val):
        got = oracle.pow_half(int(k))
        assert got == v and got != math.sqrt(k)
    rng = np.random.RandomState(0)
    exc_set = set(exc.tolist())
    for k in rng.randint(0, 2_000_000, 3000):
        if int(k) not in exc_set:
            assert oracle.pow_half(int(k)) == math.sqrt(k)
    assert oracle.pow_half(0) == 0.0


def test_mt19937_uniforms_and_choice(golden):
    z = golden("numerics")
    for s, us in zip(z["mt_seeds"], z["mt_uniforms"]):
        for k, u in enumerate(us):
            assert oracle.seed_uniform(int(s), k) == u
    for s, p, idx in zip(z["mt_seeds"], z["choice_p"], z["choice_idx"]):
        got = [oracle.choice(p, oracle.seed_uniform(int(s) + 1000, k)) for k in range(len(idx))]
        assert got == idx.tolist()


@pytest.mark.parametrize("name", ["c4", "c5_9x9", "nograv_5x5"])
def test_board_rules_match_reference(golden, name):
    z = golden("board_" + name)
    H, W, n, grav = int(z["height"]), int(z["width"]), int(z["n"]), bool(z["gravity"])
    games = z["game"]
    for g in np.unique(games):
        sel = games == g
        boards, status, mask, moves = oracle.board_replay(H, W, n, grav, z["move"][sel])
        np.testing.assert_array_equal(boards, z["array"][sel])
        want_status = np.where(~z["game_over"][sel], 0, np.where(z["is_null"][sel] == 1, 2, 1))
        np.testing.assert_array_equal(status, want_status)
        np.testing.assert_array_equal(mask, z["mask"][sel])
        np.testing.assert_array_equal(moves, z["moves_order"][sel])
        res = z["result"][sel]
        np.testing.assert_array_equal(np.where(status == 1, 1, np.where(status == 2, 0, -9)), res)


def test_synth_c_matches_python():
    rng = np.random.RandomState(3)
    for shape, grav in [((6, 7), True), ((9, 9), True), ((5, 5), False)]:
        for _ in range(200):
            b = rng.randint(-1, 2, shape).astype(np.int8)
            p, v = oracle.synth_probe(b, grav)
            own, opp = synth.masks_from_array(b, shape[1])
            A = shape[1] if grav else shape[0] * shape[1]
            wp, wv = synth.synth_eval(own, opp, A)
            np.testing.assert_array_equal(p, np.asarray(wp, np.float32))
            assert v == wv


def check_game_against_golden(z, g, got):
    """Compare one game's per-ply record with fixture game index g (bitwise)."""
    lens = z["game_len"]
    off = int(lens[:g].sum())
    T = int(lens[g])
    sl = slice(off, off + T)
    assert got["T"] == T
    np.testing.assert_array_equal(got["moves"], z["moves"][sl])
    np.testing.assert_array_equal(got["greedy"], z["greedy"][sl])
    np.testing.assert_array_equal(got["n_edges"], z["n_edges"][sl])
    np.testing.assert_array_equal(got["edge_action"], z["edge_action"][sl])
    np.testing.assert_array_equal(got["edge_n"], z["edge_n"][sl])
    np.testing.assert_array_equal(got["edge_prior"].view(np.uint64), z["edge_prior"][sl].view(np.uint64))
    np.testing.assert_array_equal(got["edge_w"].view(np.uint64), z["edge_w"][sl].view(np.uint64))
    np.testing.assert_array_equal(got["policy"].view(np.uint64), z["policy"][sl].view(np.uint64))
    np.testing.assert_array_equal(got["rewards"], z["reward"][sl])
    if "states" in got:
        np.testing.assert_array_equal(got["states"], z["state"][sl])
    else:
        np.testing.assert_array_equal(oracle.full_state(got["boards"]), z["state"][sl])
    if "expansions" in got:
        assert got["expansions"] == z["expansions"][g]


@pytest.mark.parametrize("name", MCTS_FIXTURES)
def test_oracle_selfplay_matches_reference(golden, name):
    z = golden("mcts_" + name)
    H, W, n, grav, S = (int(z[k]) for k in ("height", "width", "n", "gravity", "sims"))
    for g, seed in enumerate(z["seed"]):
        got = oracle.play_game(H, W, n, bool(grav), S, int(seed))
        check_game_against_golden(z, g, got)


NOISE_FIXTURES = ["c4_s25_noise", "c4_s100_noise", "c5_9x9_s50_noise", "nograv_5x5_s25_noise"]


def noise_of(z):
    return (float(z["dirichlet_alpha"]), float(z["dirichlet_ratio"])) if bool(z["dirichlet_noise"]) else None


@pytest.mark.parametrize("name", NOISE_FIXTURES)
def test_oracle_selfplay_with_dirichlet_noise_matches_reference(golden, name):
    """the reference's root Dirichlet noise (mcts.py:70-85,
    enable_dirichlet_noise = True) -- every root selection draws
    np.random.dirichlet(0.03 * ones(k)) from the game's stream and mixes it
    into the priors at 0.25 -- restated in the C oracle; visit counts, W,
    priors, moves and policies bitwise the reference's (fixtures generated by
    the reference itself, tests/golden/make_golden.py)."""
    z = golden("mcts_" + name)
    assert bool(z["dirichlet_noise"])
    H, W, n, grav, S = (int(z[k]) for k in ("height", "width", "n", "gravity", "sims"))
    for g, seed in enumerate(z["seed"]):
        got = oracle.play_game(H, W, n, bool(grav), S, int(seed), noise=noise_of(z))
        check_game_against_golden(z, g, got)


def test_oracle_dirichlet_is_numpys_legacy_sampler():
    """The oracle's Dirichlet restatement draws exactly what numpy's legacy
    RandomState.dirichlet draws from the same seed (this interpreter's numpy
    keeps the legacy sampler for RandomState; both call libm log / pow)."""
    for seed, k, alpha in ((0, 7, 0.03), (5, 7, 0.03), (99, 9, 0.03), (7, 25, 0.03), (3, 4, 0.5), (11, 3, 1.0)):
        rs = np.random.RandomState(seed)
        ref = np.stack([rs.dirichlet(np.ones(k) * alpha) for _ in range(200)])
        got = oracle.dirichlet_draws(seed, alpha, k, 200)
        np.testing.assert_array_equal(got.view(np.uint64), ref.view(np.uint64))


def test_table_evaluator_replays_synthetic():
    """The replay (table) evaluator gives the same game as the one it recorded."""
    rec = []

    def cb(board):
        own, opp = synth.masks_from_array(board, board.shape[1])
        p, v = synth.synth_eval(own, opp, 7)
        rec.append((board.copy(), p, v))
        return np.asarray(p, np.float32), v

    a = oracle.play_game(6, 7, 4, True, 30, 77, evaluator="callback", callback=cb)
    b0 = oracle.play_game(6, 7, 4, True, 30, 77)
    np.testing.assert_array_equal(a["edge_n"], b0["edge_n"])
    boards = np.stack([r[0] for r in rec])
    table = oracle.EvalTable(oracle.board_keys(boards), np.stack([r[1] for r in rec]),
                             np.asarray([r[2] for r in rec]))
    b = oracle.play_game(6, 7, 4, True, 30, 77, evaluator="table", table=table)
    assert table.misses() == 0
    np.testing.assert_array_equal(a["edge_w"], b["edge_w"])
    np.testing.assert_array_equal(a["moves"], b["moves"])
