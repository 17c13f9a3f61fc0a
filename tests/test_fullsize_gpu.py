"""Self-play at BASELINE.json's full single-GPU sizes, checked through
size-independent properties plus bit-exact oracle replay of sampled games.

configs[1]: Connect-4, 100 sims/move, 4096 concurrent games, random-init
network (the bench workload, with and without its 2^25-entry transposition
cache).  configs[2]: Connect-5 on 9x9, 200 sims/move, 8192 concurrent games.
configs[3]: one GPU's shard of 32768 Connect-4 games at 400 sims/move (the
last of 8 ranks: games 28672..32767, seeds base + game index).  configs[4]: chess, 800 sims/move, 256 concurrent games per GPU
(2048 across 8), random-init network, games capped at 3 plies so the test
finishes in seconds.  The small-size parity tests (test_engine_gpu.py,
test_chess_selfplay_gpu.py) pin the arithmetic; these pin that nothing
changes at the sizes the bench runs (arena sizing and subtree reclamation,
queue chunking, cache pressure, slot counts past one workgroup grid).
"""
import numpy as np
import pytest

import chess_oracle as C
import keras_ref
import oracle
from custom_alphazero import engine as az
from test_chess_selfplay_gpu import _compare
from test_engine_gpu import NET_TOL, make_net_engine, selfplay_games

pytestmark = pytest.mark.gpu

C4 = dict(H=6, W=7, n=4, grav=True, S=100, slots=4096)
C4_SEED = 4242
GREEDY_PLY = 8  # ConfigSelfPlay.index_move_greedy (reference config.py)


@pytest.fixture(scope="module")
def c4_games():
    out = {}
    for cache_log2 in (0, 25):
        # the cached run also reclaims left subtrees (compact, as bench.py runs): its games
        # equal the plain run's bit for bit (test_c4_fullsize_cache_is_transparent)
        eng, _ = make_net_engine(**C4, seed=11, cache_log2=cache_log2, compact=cache_log2 > 0)
        out[cache_log2] = (eng, selfplay_games(eng, 0, C4["slots"], base_seed=C4_SEED))
    yield out
    for eng, _ in out.values():
        eng.close()


def check_rules_and_policies(games, H, W, n):
    """Every game replays legally on the oracle rules: board before each move,
    terminal status only at the end, result = the last mover's outcome;
    policies normalised, supported on legal columns, one-hot on the move from
    ply 8."""
    for g, got in enumerate(games):
        T = got["T"]
        assert 2 * n - 1 <= T <= H * W, (g, T)
        boards, status, mask, _ = oracle.board_replay(H, W, n, True, got["moves"])
        assert (status[:-1] == 0).all() and status[-1] in (1, 2), (g, status)
        assert not got["boards"][0].any()  # every game starts on the empty board
        np.testing.assert_array_equal(got["boards"][1:], boards[:-1])
        assert got["rewards"][-1] == (1 if status[-1] == 1 else 0)
        legal = np.vstack([np.ones((1, W), bool), mask[:-1]])
        pol = got["policy"]
        assert (pol >= 0).all() and np.allclose(pol.sum(axis=1), 1.0, rtol=0, atol=1e-12), g
        assert not (pol[~legal] != 0).any(), g
        assert (pol[np.arange(T), got["moves"]] > 0).all(), g
        if T > GREEDY_PLY:
            tail = pol[GREEDY_PLY:]
            assert ((tail == 0) | (tail == 1)).all() and (tail.sum(axis=1) == 1).all(), g
            np.testing.assert_array_equal(tail.argmax(axis=1), got["moves"][GREEDY_PLY:])


def replay_on_oracle(eng, got, H, W, n, S, seed):
    """One engine game == the oracle's MCTS (reference self_play.py:37-82)
    driven by the engine's own batch-1 network outputs."""
    cache = {}

    def cb(board):
        key = board.tobytes()
        if key not in cache:
            p, v = eng.forward(oracle.full_state(board[None]))
            cache[key] = (p[0], float(v[0]))
        return cache[key]

    ref = oracle.play_game(H, W, n, True, S, seed, evaluator="callback", callback=cb)
    assert got["T"] == ref["T"]
    np.testing.assert_array_equal(got["moves"], ref["moves"])
    np.testing.assert_array_equal(got["policy"].view(np.uint64), ref["policy"].view(np.uint64))
    assert got["expansions"] == ref["expansions"]


def test_c4_fullsize_rules_and_policies(c4_games):
    check_rules_and_policies(c4_games[25][1], C4["H"], C4["W"], C4["n"])


def test_c4_fullsize_cache_is_transparent(c4_games):
    """The transposition cache at the bench size changes nothing: same moves,
    policies (bitwise) and expansion counts for all 4096 games."""
    a, b = c4_games[0][1], c4_games[25][1]
    for g, (x, y) in enumerate(zip(a, b)):
        assert x["T"] == y["T"] and x["expansions"] == y["expansions"], g
        np.testing.assert_array_equal(x["moves"], y["moves"])
        np.testing.assert_array_equal(x["policy"].view(np.uint64), y["policy"].view(np.uint64))


@pytest.mark.parametrize("g", [0, 1777, 4095])
def test_c4_fullsize_game_replays_on_oracle(c4_games, g):
    """Sampled games of the 4096 replay bit for bit through the oracle's MCTS
    (reference self_play.py:37-82) driven by the engine's own batch-1 network
    outputs."""
    eng, games = c4_games[25]
    replay_on_oracle(eng, games[g], C4["H"], C4["W"], C4["n"], C4["S"], C4_SEED + g)


def playout_boards(rng, k, H, W):
    """k gravity positions reached by random play from the empty board (0 to
    H*W - 1 plies, the side to move as +1), as int8 [k, H, W]."""
    b = np.zeros((k, H, W), np.int8)
    plies = rng.randint(0, H * W, k)
    for t in range(H * W - 1):
        live = np.nonzero(plies > t)[0]
        if not len(live):
            break
        b[live] *= -1  # the mover's stones become the opponent's
        height = (b[live] != 0).sum(axis=1)  # stones per column
        for i, row in zip(live, height):
            cols = np.nonzero(row < H)[0]
            c = cols[rng.randint(len(cols))]
            b[i, H - 1 - row[c], c] = -1  # the stone of the player who just moved
    return b


def forward_vs_keras(H, W, n, x, seed):
    eng, w = make_net_engine(H, W, n, True, slots=len(x), seed=seed)
    try:
        p, v = eng.forward(x)
    finally:
        eng.close()
    rp, rv = keras_ref.forward(w, x, depth=4)
    assert np.abs(p - rp).max() < NET_TOL, np.abs(p - rp).max()
    assert np.abs(v - rv).max() < NET_TOL, np.abs(v - rv).max()


@pytest.mark.parametrize("B", [672, 4096])
def test_c4_forward_at_bench_batches_matches_keras(c4_games, B):
    """The tower at the bench's launch sizes (672 boards: one lane's live
    batch in bench.py; 4096: 1366 tiles, more than five per CU) on positions
    the bench workload's own games reach (every ply of the 4096 self-play
    games above), within NET_TOL of the float64 Keras restatement -- not only
    the 37-board random fills of test_engine_gpu.py."""
    pos = np.concatenate([g["boards"] for g in c4_games[25][1]])
    rng = np.random.RandomState(B)
    forward_vs_keras(6, 7, 4, oracle.full_state(pos[rng.choice(len(pos), B, replace=False)]), seed=11)


def test_c5_9x9_forward_at_bench_batch_matches_keras():
    """configs[2]'s launch size (3443 boards: one lane's live batch in
    bench.py, two 9x9 boards per 192-row tile) on random-playout positions,
    within NET_TOL of the float64 Keras restatement."""
    rng = np.random.RandomState(9)
    forward_vs_keras(9, 9, 5, oracle.full_state(playout_boards(rng, 3443, 9, 9)), seed=13)


@pytest.mark.parametrize("cfg", [
    dict(H=9, W=9, n=5, S=200, slots=8192, first=0, replay=(8191,)),        # configs[2]
    dict(H=6, W=7, n=4, S=400, slots=4096, first=7 * 4096, replay=(4095,)),  # configs[3], rank 7
    dict(H=6, W=7, n=4, S=400, slots=16384, first=16384, replay=(0, 16383)),  # configs[3] over 2 GPUs, rank 1
], ids=["c5_9x9_s200_8192", "c4_s400_shard7", "c4_s400_2gpu_shard1"])
@pytest.mark.timeout(400)  # configs[2] plays ~80M expansions (about 90 s)
def test_connect_n_fullsize_configs(cfg):
    """BASELINE configs[2] and one rank's shard of configs[3] at full size --
    8 ranks (4096 games each) and 2 ranks (16384 games each, the largest
    shard configs[3] names): rules and policies for every game, sampled games
    replayed on the oracle (a shard's game i uses seed base + first + i, as
    bench.py's ranks do); the pooled arenas hold every tree (no device error)."""
    H, W, n, S = cfg["H"], cfg["W"], cfg["n"], cfg["S"]
    eng, _ = make_net_engine(H, W, n, True, S=S, slots=cfg["slots"], seed=13, cache_log2=25, compact=True)
    try:
        games = selfplay_games(eng, cfg["first"], cfg["slots"], base_seed=C4_SEED)
        st = eng.stats()
        assert st["errors"] == 0 and 0 < st["arena_pool_high"] <= st["arena_pool_edges"] // 2
        check_rules_and_policies(games, H, W, n)
        for g in cfg["replay"]:
            replay_on_oracle(eng, games[g], H, W, n, S, C4_SEED + cfg["first"] + g)
    finally:
        eng.close()


CHESS = dict(sims=800, slots=256, plies=32)
CHESS_SEED = 900


@pytest.fixture(scope="module")
def chess_games():
    from custom_alphazero.model.weights import init_weights, weight_spec
    w = init_weights(weight_spec(8, 8, 1880, in_channels=118), seed=5)
    eng = az.ChessEngine(mcts_iterations=CHESS["sims"], slots=CHESS["slots"],
                         evaluator=az.EVAL_NETWORK, max_plies=CHESS["plies"])
    eng.set_weights(w.items())
    st = eng.selfplay_run(0, CHESS["slots"], CHESS_SEED)
    assert st["errors"] == 0 and st["games_done"] == CHESS["slots"]
    yield eng, eng.selfplay_results()
    eng.close()


def check_chess_games(r, n_games, plies):
    """Positions chain through Board.play on the oracle rules, each move is
    legal, each root policy covers exactly the legal moves (in the 1880-action
    space) and is normalised; games end at the ply cap or earlier with a
    terminal position."""
    all_mv = C.all_moves()
    start = C.from_fen()
    for g in range(n_games):
        T = int(r["lengths"][g])
        assert T == plies and r["terminations"][g] == 5 or T < plies and r["terminations"][g] != 5, g
        pos = start
        for t in range(T):
            assert r["positions"][g, t].tobytes() == pos.tobytes(), (g, t)
            mv = int(r["moves"][g, t])
            assert mv in set(C.legal_moves(pos).tolist()), (g, t)
            legal = np.flatnonzero(C.legal_mask(pos, all_mv))
            k = int(r["policy_n"][g, t])
            acts = r["policy_actions"][g, t, :k]
            np.testing.assert_array_equal(np.sort(acts), legal)
            probs = r["policy_probs"][g, t, :k]
            assert (probs >= 0).all() and abs(probs.sum() - 1.0) < 1e-12, (g, t)
            assert probs[list(all_mv[acts]).index(mv)] > 0, (g, t)
            pos = C.play_canonical(pos, mv)
        assert r["expansions"][g] >= T, g


@pytest.mark.timeout(400)
def test_chess_fullsize_rules_and_policies(chess_games):
    """All 256 games at 800 sims/move (BASELINE configs[4]'s per-GPU shard)
    over 32 plies (the kept subtree compacted every move): positions, legal
    moves and root policies checked ply by ply on the oracle rules."""
    _, r = chess_games
    check_chess_games(r, CHESS["slots"], CHESS["plies"])
    assert (r["lengths"][:CHESS["slots"]] <= CHESS["plies"]).all()
    # random-init play mates early in a few games (the terminal positions are
    # checked above); most run to the cap
    assert (r["lengths"][:CHESS["slots"]] == CHESS["plies"]).mean() > 0.75


CHESS_LONG = dict(sims=800, slots=32, plies=64)


@pytest.mark.timeout(300)
def test_chess_long_games_at_800_sims():
    """configs[4]'s 800 sims/move over 64 plies (the subtree kept across
    moves grows with the search, compaction every move): rules and policies
    for all 32 games, games 0 and 31 replayed bit for bit on the oracle."""
    from custom_alphazero.model.weights import init_weights, weight_spec
    w = init_weights(weight_spec(8, 8, 1880, in_channels=118), seed=6)
    eng = az.ChessEngine(mcts_iterations=CHESS_LONG["sims"], slots=CHESS_LONG["slots"],
                         evaluator=az.EVAL_NETWORK, max_plies=CHESS_LONG["plies"])
    try:
        eng.set_weights(w.items())
        st = eng.selfplay_run(0, CHESS_LONG["slots"], CHESS_SEED)
        assert st["errors"] == 0 and st["games_done"] == CHESS_LONG["slots"]
        r = eng.selfplay_results()
        check_chess_games(r, CHESS_LONG["slots"], CHESS_LONG["plies"])

        def cb(pos, initial):
            x = C.full_state(*C.reference_history(pos, bool(initial)), pos)[None].astype(np.float32)
            p, v = eng.forward(x)
            return p[0], float(v[0])

        for g in (0, CHESS_LONG["slots"] - 1):
            ref = C.play_game(CHESS_LONG["sims"], CHESS_SEED + g, CHESS_LONG["plies"], callback=cb)
            _compare(r, g, ref, "long")
    finally:
        eng.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("g", [0, 255])
def test_chess_fullsize_game_replays_on_oracle(chess_games, g):
    """Games of the 256 replay bit for bit through the chess oracle's MCTS
    with the engine's own batch-1 network outputs (800 sims/move)."""
    eng, r = chess_games

    def cb(pos, initial):
        x = C.full_state(*C.reference_history(pos, bool(initial)), pos)[None].astype(np.float32)
        p, v = eng.forward(x)
        return p[0], float(v[0])

    ref = C.play_game(CHESS["sims"], CHESS_SEED + g, CHESS["plies"], callback=cb)
    _compare(r, g, ref, "fullsize")


CHESS_END = dict(sims=800, slots=8, plies=512)


@pytest.mark.timeout(600)
def test_chess_games_to_termination_at_800_sims():
    """configs[4]'s 800 sims/move played from the opening
    to the end -- 8 games, every one finishing by the rules (checkmate,
    stalemate, insufficient material, the 75-move rule) or at the 512-ply
    cap the reference lacks -- with rules and policies checked at every ply
    and the shortest rule-terminated game replayed bit for bit on the oracle
    (its network outputs: the engine's own batch-1 forward)."""
    from custom_alphazero.model.weights import init_weights, weight_spec
    w = init_weights(weight_spec(8, 8, 1880, in_channels=118), seed=7)
    eng = az.ChessEngine(mcts_iterations=CHESS_END["sims"], slots=CHESS_END["slots"],
                         evaluator=az.EVAL_NETWORK, max_plies=CHESS_END["plies"])
    try:
        eng.set_weights(w.items())
        st = eng.selfplay_run(0, CHESS_END["slots"], CHESS_SEED)
        assert st["errors"] == 0 and st["games_done"] == CHESS_END["slots"]
        r = eng.selfplay_results()
        check_chess_games(r, CHESS_END["slots"], CHESS_END["plies"])
        lengths = r["lengths"][:CHESS_END["slots"]]
        terms = r["terminations"][:CHESS_END["slots"]]
        ended = [g for g in range(CHESS_END["slots"]) if terms[g] != 5]
        assert ended, (lengths.tolist(), terms.tolist())  # some game ends by the rules
        print(f"chess to termination: lengths {lengths.tolist()}, terminations {terms.tolist()}")

        def cb(pos, initial):
            x = C.full_state(*C.reference_history(pos, bool(initial)), pos)[None].astype(np.float32)
            p, v = eng.forward(x)
            return p[0], float(v[0])

        g = min(ended, key=lambda k: int(lengths[k]))
        ref = C.play_game(CHESS_END["sims"], CHESS_SEED + g, CHESS_END["plies"], callback=cb)
        _compare(r, g, ref, "to-termination")
    finally:
        eng.close()
