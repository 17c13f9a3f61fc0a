"""BASELINE configs[4] chess games played to their end on the GPU: 800
simulations per move, the 128-filter 4-block network, no ply cap short of
the engine's 512 (the reference's games end only by the rules:
custom_alphazero/chess/board.py:58-73 via python-chess's outcome()).

* synthetic evaluator: eight games bitwise against the chess oracle's MCTS
  (oracle/chess_oracle.c, the reference's mcts.py:86-222 restated) --
  every root position, move, MCTS.play policy, expansion count,
  termination and result;
* network evaluator: eight games checked move by move against the oracle's
  rules (each move legal, each next root the reference's
  Board.play(keep_same_player=True) of the last, each policy a distribution
  over exactly the root's legal moves, each ending python-chess's outcome()
  of the final position or the cap), and the first plies of one game
  replayed through the oracle's MCTS with the engine's own batch-1 network
  outputs as its evaluator (bitwise)."""
import numpy as np
import pytest

import chess_oracle as C

pytestmark = pytest.mark.gpu
SIMS, PLIES, GAMES = 800, 512, 8


def _legal_actions(pos, index):
    return np.sort(np.array([index[int(m)] for m in C.legal_moves(pos)], np.int64))


def test_chess_configs4_games_synthetic_match_oracle():
    from custom_alphazero import engine as az
    from test_chess_selfplay_gpu import _compare
    eng = az.ChessEngine(mcts_iterations=SIMS, slots=GAMES, evaluator=az.EVAL_SYNTHETIC, max_plies=PLIES,
                         index_move_greedy=8, lanes=2)
    st = eng.selfplay_run(0, GAMES, 4000)
    r = eng.selfplay_results()
    eng.close()
    assert st["errors"] == 0 and st["games_done"] == GAMES
    ends = set()
    for g in range(GAMES):
        ref = C.play_game(SIMS, 4000 + g, PLIES, greedy_ply=8)
        _compare(r, g, ref, "synthetic-800")
        ends.add(int(ref["termination"]))
    assert ends - {5}, "every game hit the cap: no rules ending was exercised"


def test_chess_configs4_games_network_follow_the_rules():
    from custom_alphazero import engine as az
    from custom_alphazero.model.weights import init_weights, weight_spec
    from test_chess_selfplay_gpu import _compare
    w = init_weights(weight_spec(8, 8, 1880, in_channels=118), seed=11, randomize_bn=True)
    eng = az.ChessEngine(mcts_iterations=SIMS, slots=GAMES, evaluator=az.EVAL_NETWORK, max_plies=PLIES,
                         index_move_greedy=8)
    eng.set_weights(w.items())
    st = eng.selfplay_run(0, GAMES, 900)
    r = eng.selfplay_results()
    assert st["errors"] == 0 and st["games_done"] == GAMES
    index = {int(m): i for i, m in enumerate(C.all_moves())}
    for g in range(GAMES):
        T = int(r["lengths"][g])
        assert 0 < T <= PLIES
        pos = C.from_fen()
        for t in range(T):
            assert r["positions"][g, t].tobytes() == np.array([pos], C.POS_DTYPE).tobytes(), (g, t)
            legal = C.legal_moves(pos)
            mv = int(r["moves"][g, t])
            assert mv in set(int(m) for m in legal), (g, t, C.uci(mv))
            n = int(r["policy_n"][g, t])
            acts = np.asarray(r["policy_actions"][g, t, :n], np.int64)
            assert np.array_equal(np.sort(acts), _legal_actions(pos, index)), (g, t)
            p = np.asarray(r["policy_probs"][g, t, :n], np.float64)
            assert (p >= 0).all() and abs(p.sum() - 1.0) < 1e-12 and p[acts == index[mv]][0] > 0, (g, t)
            pos = C.play_canonical(pos, mv)
        term = C.outcome(pos)
        if term == 0:
            assert T == PLIES and r["terminations"][g] == 5, (g, T)
        else:
            assert r["terminations"][g] == term, (g, term)
        assert r["results"][g] == (1 if term == 1 else 0), g

    # the first plies of game 0 through the oracle's MCTS, evaluated by the
    # engine's own network one board at a time (batch invariant: the chess
    # forward test checks it)
    def cb(pos, initial):
        x = C.full_state(*C.reference_history(pos, bool(initial)), pos)[None].astype(np.float32)
        p, v = eng.forward(x)
        return p[0], float(v[0])

    k = min(6, int(r["lengths"][0]))
    ref = C.play_game(SIMS, 900, k, greedy_ply=8, callback=cb)
    assert ref["T"] == k
    for t in range(k):
        assert int(r["moves"][0, t]) == int(ref["moves"][t]), t
        n = int(ref["policy_n"][t])
        assert np.array_equal(r["policy_probs"][0, t, :n].view(np.uint64), ref["policy_probs"][t, :n].view(np.uint64)), t
    eng.close()
