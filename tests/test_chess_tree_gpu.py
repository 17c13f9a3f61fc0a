"""MCTS tree API on chess boards (az_chess_tree_*, mcts.MCTS with a chess
Board) against the chess oracle's MCTS object (oracle/chess_oracle.c
orc_chess_tree_*, restating mcts/mcts.py:86-222): root edges after every
search (move order, priors and W bitwise, visit counts, child expansions),
play's move and policy, tree reuse across moves, greedy and deterministic
play, several roots at once, roots other than the start position (whose
deepcopied history is [0 x 7, start-position state])."""
import numpy as np
import pytest

import chess_oracle as C

pytestmark = pytest.mark.gpu

ROOTS = [
    C.START_FEN,
    "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1",
    "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1",
    "r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1",
    "rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8",
    "6k1/5ppp/8/8/8/8/5PPP/R5K1 w - - 0 30",  # back-rank mate in one
]


def _engine(slots, evaluator, sims=64, lanes=1):
    from custom_alphazero import engine as az
    return az.ChessEngine(mcts_iterations=sims, slots=slots, evaluator=evaluator, max_plies=64,
                          lanes=lanes, arena_edges=50_000)


def _root_edges(eng, slot):
    t = eng.tree_export(slot)
    f, k = t["root_first"], t["root_n"]
    sl = slice(f, f + k)
    return dict(moves=t["moves"][sl], prior=t["prior"][sl], n=t["n"][sl], w=t["w"][sl],
                child_n=t["child_n"][sl])


def _check_root(eng, slot, ref, tag):
    got, want = _root_edges(eng, slot), ref.root()
    assert len(got["moves"]) == len(want["moves"]), tag
    np.testing.assert_array_equal(got["moves"], want["moves"].astype(np.int32))
    np.testing.assert_array_equal(got["prior"].view(np.uint64), want["prior"].view(np.uint64))
    np.testing.assert_array_equal(got["n"], want["n"])
    np.testing.assert_array_equal(got["w"].view(np.uint64), want["w"].view(np.uint64))
    np.testing.assert_array_equal(got["child_n"], want["child_n"])


def _run(eng, trees, plan, seed):
    """plan: list of (sims, greedy, deterministic) per move, applied to every slot."""
    rng = np.random.RandomState(seed)
    S = len(trees)
    for step, (sims, greedy, det) in enumerate(plan):
        eng.tree_search(sims)
        for tr in trees:
            tr.search(sims)
        for s, tr in enumerate(trees):
            _check_root(eng, s, tr, (step, s))
        u = rng.random_sample(S)
        out = eng.tree_play(u, greedy=greedy, deterministic=det)
        for s, tr in enumerate(trees):
            mv, oc, pa, pp = tr.play(u[s], greedy, det)
            assert out["moves"][s] == mv and out["status"][s] == oc, (step, s)
            k = int(out["policy_n"][s])
            assert k == len(pa)
            np.testing.assert_array_equal(out["policy_actions"][s, :k], pa)
            np.testing.assert_array_equal(out["policy_probs"][s, :k].view(np.uint64), pp.view(np.uint64))
        # the reused subtree is the oracle's chosen child
        for s, tr in enumerate(trees):
            if out["status"][s] == 0:
                _check_root(eng, s, tr, ("reuse", step, s))


PLAN = [(40, False, False), (25, False, False), (1, False, False), (30, True, False),
        (20, False, True), (10, True, True)]


@pytest.mark.parametrize("lanes", [1, 2])
def test_chess_tree_synthetic_matches_oracle(lanes):
    from custom_alphazero import engine as az
    roots = [C.from_fen(f) for f in ROOTS[:5]]
    eng = _engine(len(roots), az.EVAL_SYNTHETIC, lanes=lanes)
    eng.tree_reset(np.arange(len(roots)), np.array(roots, C.POS_DTYPE))
    trees = [C.Tree(r) for r in roots]
    _run(eng, trees, PLAN, seed=11 + lanes)
    st = eng.stats()
    assert st["expansions"] == sum(t.expansions for t in trees)
    eng.close()


def test_chess_tree_release_and_partial_reset():
    """Idle slots are skipped by search and play; a reset slot starts over
    while the others keep their trees."""
    from custom_alphazero import engine as az
    roots = [C.from_fen(ROOTS[1]), C.from_fen(ROOTS[4])]
    eng = _engine(2, az.EVAL_SYNTHETIC)
    eng.tree_reset([0, 1], np.array(roots, C.POS_DTYPE))
    eng.tree_search(12)
    before = _root_edges(eng, 1)
    eng.tree_release([1])
    eng.tree_search(5)
    out = eng.tree_play(np.array([0.5, 0.5]))
    assert out["moves"][1] == -1 and out["moves"][0] >= 0
    after = _root_edges(eng, 1)
    np.testing.assert_array_equal(before["n"], after["n"])
    t0 = C.Tree(roots[0])
    t0.search(17)
    t0.play(0.5)
    _check_root(eng, 0, t0, "slot 0")
    new_root = C.play_canonical(C.from_fen(), C.legal_moves(C.from_fen())[3])
    eng.tree_reset([1], np.array([new_root], C.POS_DTYPE))
    eng.tree_search(9)
    t1 = C.Tree(new_root)
    t1.search(9)
    _check_root(eng, 1, t1, "slot 1 reset")
    t0.search(9)  # slot 0 stayed active and searched too
    _check_root(eng, 0, t0, "slot 0 kept")
    eng.close()


def test_chess_tree_terminal_root_and_mate_in_one():
    from custom_alphazero import engine as az
    eng = _engine(1, az.EVAL_SYNTHETIC)
    root = C.from_fen(ROOTS[5])
    eng.tree_reset([0], np.array([root], C.POS_DTYPE))
    tr = C.Tree(root)
    _run(eng, [tr], [(200, False, True)], seed=0)
    eng.close()
    # a checkmated root: search backs up nothing, play has no edge to choose
    mated = C.from_fen("rnb1kbnr/pppp1ppp/8/4p3/6Pq/5P2/PPPPP2P/RNBQKBNR w KQkq - 1 3")
    eng = _engine(1, az.EVAL_SYNTHETIC)
    eng.tree_reset([0], np.array([mated], C.POS_DTYPE))
    eng.tree_search(5)
    assert _root_edges(eng, 0)["moves"].size == 0
    with pytest.raises(az.AzError, match="play-before-search"):
        eng.tree_play(np.array([0.1]))
    # that error leaves the engine usable: a new root searches and plays
    root = C.from_fen(ROOTS[2])
    eng.tree_reset([0], np.array([root], C.POS_DTYPE))
    tr = C.Tree(root)
    _run(eng, [tr], [(12, False, False)], seed=3)
    eng.close()


@pytest.fixture(scope="module")
def chess_net_tree():
    from custom_alphazero import engine as az
    from custom_alphazero.model.weights import init_weights, weight_spec
    w = init_weights(weight_spec(8, 8, 1880, in_channels=118), seed=9)
    eng = _engine(2, az.EVAL_NETWORK, sims=32)
    eng.set_weights(w.items())
    yield eng
    eng.close()


def test_chess_tree_network_matches_oracle(chess_net_tree):
    """Network evaluator: the oracle, fed the engine's batch-1 outputs on the
    reference's full_state (root: [0 x 7, start state] even for a
    non-start root), reproduces both trees bit for bit."""
    eng = chess_net_tree

    def cb(pos, initial):
        x = C.full_state(*C.reference_history(pos, bool(initial)), pos)[None].astype(np.float32)
        p, v = eng.forward(x)
        return p[0], float(v[0])

    roots = [C.from_fen(ROOTS[0]), C.from_fen(ROOTS[1])]
    eng.tree_reset([0, 1], np.array(roots, C.POS_DTYPE))
    trees = [C.Tree(r, callback=cb) for r in roots]
    _run(eng, trees, [(24, False, False), (12, False, False), (8, True, False)], seed=5)


def test_chess_mcts_api_matches_oracle():
    """mcts.MCTS with a chess Board (the reference's object API): search,
    play(return_details) with the global numpy stream, tree views."""
    from custom_alphazero.chess.board import Board
    from custom_alphazero.chess.utils import get_all_possible_moves
    from custom_alphazero.config import ConfigSelfPlay
    from custom_alphazero.mcts.mcts import MCTS, ChessMCTS, SyntheticEvaluator
    moves = get_all_possible_moves()
    fen = ROOTS[4].split()[0]
    saved = ConfigSelfPlay.mcts_iterations
    try:
        ConfigSelfPlay.mcts_iterations = 30
        board = Board(board_fen=fen)
        m = MCTS(board=board, all_possible_moves=moves, concurrency=False, plays_inferences={},
                 model=SyntheticEvaluator())
    finally:
        ConfigSelfPlay.mcts_iterations = saved
    assert isinstance(m, ChessMCTS)
    tr = C.Tree(board._pos)
    np.random.seed(123)
    rng = np.random.RandomState(123)
    for step in range(4):
        m.search(30)
        tr.search(30)
        want = tr.root()
        root = m.current_root
        assert [e.action.code for e in root.edges] == want["moves"].tolist()
        assert [e.visit_count for e in root.edges] == want["n"].tolist()
        parent, child, policy, move = m.play(greedy=step == 3, return_details=True)
        mv, oc, pa, pp = tr.play(rng.random_sample(), step == 3, False)
        assert move.code == mv
        dense = np.zeros(len(moves))
        dense[pa.astype(np.int64)] = pp
        np.testing.assert_array_equal(policy, dense)
        assert parent.shape == child.shape == (8, 8, 118)
        assert m.board.is_game_over() == (oc != 0)
        if oc:
            break
    assert step >= 2
    if m.board.is_game_over():
        m.search(5)  # a finished board: nothing to search
        with pytest.raises(RuntimeError, match="finished game"):
            m.play()
    # the deepcopied root's history quirk reaches play()'s parent state too
    fresh = MCTS(board=Board(board_fen=fen), all_possible_moves=moves, model=SyntheticEvaluator())
    x = fresh.board.full_state
    ref = C.full_state(*C.reference_history(board._pos, True), board._pos)
    np.testing.assert_array_equal(x, ref)


def test_chess_mcts_api_with_model_matches_oracle():
    """mcts.MCTS on a chess Board with a chess PolicyValueModel (input
    (8, 8, 118), 1880 actions): the oracle's MCTS object, fed the model's own
    outputs on the reference's full_state, gives the same root edges and
    moves (a non-start root: history [0 x 7, start state])."""
    from custom_alphazero.chess.board import Board
    from custom_alphazero.chess.utils import get_all_possible_moves
    from custom_alphazero.config import ConfigSelfPlay
    from custom_alphazero.mcts.mcts import MCTS
    from custom_alphazero.model.policy_value import PolicyValueModel
    model = PolicyValueModel(input_dim=(8, 8, 118), action_space=1880, seed=4)
    moves = get_all_possible_moves()
    board = Board(board_fen=ROOTS[1].split()[0])
    saved = ConfigSelfPlay.mcts_iterations
    try:
        ConfigSelfPlay.mcts_iterations = 20
        m = MCTS(board=board, all_possible_moves=moves, concurrency=False, plays_inferences={}, model=model)
    finally:
        ConfigSelfPlay.mcts_iterations = saved

    def cb(pos, initial):
        x = C.full_state(*C.reference_history(pos, bool(initial)), pos)[None].astype(np.float32)
        p, v = model(x)
        return p.numpy()[0], float(v.numpy()[0, 0])

    tr = C.Tree(board._pos, callback=cb)
    np.random.seed(7)
    rng = np.random.RandomState(7)
    for step in range(3):
        m.search(20)
        tr.search(20)
        want = tr.root()
        root = m.current_root
        assert [e.action.code for e in root.edges] == want["moves"].tolist()
        assert [e.visit_count for e in root.edges] == want["n"].tolist()
        assert np.array_equal(np.array([e.prior for e in root.edges]).view(np.uint64),
                              want["prior"].view(np.uint64))
        _, _, policy, move = m.play(return_details=True)
        mv, oc, pa, pp = tr.play(rng.random_sample())
        assert move.code == mv
        if oc:
            break
