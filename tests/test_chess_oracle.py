"""Chess oracle (oracle/chess_oracle.c) pinned to known answers, plus the
host-side pieces of the chess seam that need no GPU.

Pins: published perft node counts of the standard test positions (legal move
sets + push), python-chess's documented start-position move order, the
1880-move action list of get_all_possible_moves (SURVEY.md §8 a20 hand
count).  Generation order beyond that, history planes and outcome rules are
"parity unpinned" (python-chess absent, no chess fixture in the reference).
"""
import numpy as np
import pytest

import chess_oracle as C

# chessprogramming.org "Perft Results" positions and node counts
PERFT = [
    ("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", [20, 400, 8902, 197281, 4865609]),
    ("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", [48, 2039, 97862, 4085603]),
    ("8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1", [14, 191, 2812, 43238, 674624]),
    ("r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1", [6, 264, 9467, 422333]),
    ("rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8", [44, 1486, 62379, 2103487]),
    ("r4rk1/1pp1qppp/p1np1n2/2b1p1B1/2B1P1b1/P1NP1N2/1PP1QPPP/R4RK1 w - - 0 10",
     [46, 2079, 89890, 3894594]),
]


@pytest.mark.parametrize("fen,counts", PERFT, ids=[f.split()[0][:12] for f, _ in PERFT])
def test_oracle_perft_known_answers(fen, counts):
    p = C.from_fen(fen)
    for d, expected in enumerate(counts, 1):
        assert C.perft(p, d) == expected, (fen, d)


def test_oracle_start_position_order_is_python_chess():
    # list(chess.Board().legal_moves) in python-chess: knights (g1 before b1,
    # to-squares descending), then single pushes h..a, then double pushes h..a
    expected = ["g1h3", "g1f3", "b1c3", "b1a3", "h2h3", "g2g3", "f2f3", "e2e3", "d2d3", "c2c3",
                "b2b3", "a2a3", "h2h4", "g2g4", "f2f4", "e2e4", "d2d4", "c2c4", "b2b4", "a2a4"]
    assert [C.uci(m) for m in C.legal_moves(C.from_fen())] == expected


def test_oracle_evasions_come_first_when_in_check():
    # white king e1 checked by the bishop on b4: king moves (to-squares
    # descending, d2 on the checking line excluded), then the block c2c3; no
    # castling out of check
    p = C.from_fen("4k3/8/8/8/1b6/8/2P5/R3K3 w Q - 0 1")
    assert [C.uci(m) for m in C.legal_moves(p)] == ["e1f2", "e1e2", "e1f1", "e1d1", "c2c3"]


def test_all_possible_moves_list():
    am = C.all_moves()
    assert len(am) == 1880
    keys = [(((m & 63) & 7, (m & 63) >> 3), (((m >> 6) & 63) & 7, ((m >> 6) & 63) >> 3,
             {0: "", 2: "n", 3: "b", 4: "r", 5: "q"}[m >> 12])) for m in am.tolist()]
    assert keys == sorted(keys) and len(set(keys)) == 1880
    ucis = set(C.uci(m) for m in am)
    for u in ("e1g1", "e1c1", "a7a8q", "a7b8n", "h7g8r", "b1c3", "e2e4"):
        assert u in ucis
    assert "a2a1q" not in ucis and "e7e8" in ucis  # white-only promotions; queen move e7e8


def test_libaz_action_list_matches_oracle():
    """az_chess_all_moves (host table in libaz, derived independently) ==
    the oracle's construction through the reference's procedure."""
    from custom_alphazero.chess import kernels as K
    assert np.array_equal(K.all_moves(), C.all_moves())


def test_oracle_full_state_start_position():
    p = C.from_fen()
    hist, valid = C.reference_history(p, is_root=True)
    s = C.full_state(hist, valid, p)
    assert s.shape == (8, 8, 118) and s.dtype == np.float64
    assert not s[:, :, :98].any()
    onehot = s[:, :, 98:111]
    arr = C.array(p)
    assert np.array_equal(onehot, np.eye(13)[arr])
    assert not s[:, :, 111].any()                       # repetition plane
    assert (s[:, :, 112:116] == 1).all()                # all castling rights
    assert (s[:, :, 116] == 1).all() and not s[:, :, 117].any()
    # a non-root board carries [0 x 6, start state, state]
    q = C.play_canonical(p, C.legal_moves(p)[15])  # e2e4
    hist, valid = C.reference_history(q, is_root=False)
    s2 = C.full_state(hist, valid, q)
    assert np.array_equal(s2[:, :, 84:98], s[:, :, 98:112])
    assert s2[:, :, 117].max() == 0  # pawn move zeroes the clock


def test_oracle_canonical_play_mirrors():
    p = C.from_fen()
    e4 = [m for m in C.legal_moves(p) if C.uci(m) == "e2e4"][0]
    q = C.play_canonical(p, e4)
    a = C.array(q)
    assert q["turn"] == 1 and q["fullmove_number"] == 1
    assert a[7].tolist() == [4, 2, 3, 5, 6, 3, 2, 4]        # black's pieces, now "white"
    assert a[3, 4] == -1 and a[1, 4] == 0                   # the e-pawn, seen from the other side
    assert q["ep_square"] == (5 * 8 + 4)                    # e3 flipped to e6
    assert np.array_equal(C.array(C.mirror(C.mirror(q))), a)


@pytest.mark.parametrize("fen,code", [
    ("rnb1kbnr/pppp1ppp/8/4p3/6Pq/5P2/PPPPP2P/RNBQKBNR w KQkq - 1 3", 1),   # fool's mate
    ("7k/5Q2/6K1/8/8/8/8/8 b - - 0 1", 3),                                 # stalemate
    ("8/8/8/8/8/8/8/K6k w - - 0 1", 2),                                    # K v K
    ("8/8/8/8/8/8/8/KN5k w - - 0 1", 2),                                   # KN v K
    ("8/8/8/8/8/8/8/KB4bk w - - 0 1", 0),                                  # opposite bishops
    ("8/8/8/8/8/8/R7/K6k w - - 150 90", 4),                                # 75-move rule
    ("8/8/8/8/8/8/R7/K6k w - - 149 90", 0),
])
def test_oracle_outcomes(fen, code):
    assert C.outcome(C.from_fen(fen)) == code


def test_oracle_random_playouts_are_consistent():
    pos, roots = C.random_positions(400, seed=3)
    for p in pos:
        mv = C.legal_moves(p)
        assert len(set(mv.tolist())) == len(mv)
        mask = C.legal_mask(p, C.all_moves())
        assert mask.sum() == len(mv)  # every canonical legal move is an action
