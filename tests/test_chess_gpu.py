"""GPU parity of the chess board kernels (csrc/az_chess.hip, SURVEY.md §8
a20) against the chess oracle: legal moves (set and python-chess order),
legal-move masks, outcomes, canonical play, full_state encoding, and perft on
the device at full size; plus the reference Board API on top of them."""
import os

import numpy as np
import pytest

import chess_oracle as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from custom_alphazero.chess import kernels
    return kernels


@pytest.fixture(scope="module")
def positions():
    """Canonical positions from seeded random playouts (MCTS-like: every move
    is Board.play(keep_same_player=True)) and non-canonical ones (both sides
    to move), plus the standard perft positions."""
    can, roots = C.random_positions(3000, seed=11, max_plies=300)
    raw, _ = C.random_positions(1500, seed=12, max_plies=300, canonical=False)
    from test_chess_oracle import PERFT, test_oracle_outcomes
    fens = [f for f, _ in PERFT] + [a[0] for a in test_oracle_outcomes.pytestmark[0].args[1]]
    std = np.array([C.from_fen(f) for f in fens], C.POS_DTYPE)
    pos = np.concatenate([can, raw, std])
    is_root = np.concatenate([roots, np.zeros(len(raw) + len(std), bool)])
    return pos, is_root


def test_legal_moves_order_mask_outcome_match_oracle(K, positions):
    pos, _ = positions
    moves, counts, mask, outcome = K.legal(pos)
    am = C.all_moves()
    for i, p in enumerate(pos):
        ref = C.legal_moves(p)
        assert counts[i] == len(ref), i
        assert np.array_equal(moves[i, :counts[i]], ref), (i, [C.uci(m) for m in ref])
        assert outcome[i] == C.outcome(p), i
        if p["turn"] == 1:
            assert np.array_equal(mask[i], C.legal_mask(p, am).astype(bool)), i
    # the playouts reach every termination the rules have
    assert {0, 1, 2, 3, 4} == set(outcome.tolist())


def test_play_matches_oracle(K, positions):
    pos, _ = positions
    rng = np.random.default_rng(5)
    sel, mv = [], []
    for i, p in enumerate(pos):
        ref = C.legal_moves(p)
        if len(ref):
            sel.append(i)
            mv.append(ref[rng.integers(len(ref))])
    sel, mv = np.array(sel), np.array(mv, np.uint16)
    canon = K.play(pos[sel], mv, keep_same_player=True)
    raw = K.play(pos[sel], mv, keep_same_player=False)
    for j, i in enumerate(sel):
        assert canon[j].tobytes() == C.play_canonical(pos[i], mv[j]).tobytes(), i
        assert raw[j].tobytes() == C.push(pos[i], mv[j]).tobytes(), i


def test_encode_matches_oracle_full_state(K, positions):
    pos, is_root = positions
    n = 1024
    hist = np.zeros((n, 8), C.POS_DTYPE)
    valid = np.zeros((n, 8), np.uint8)
    for i in range(n):
        h, v = C.reference_history(pos[i], bool(is_root[i]))
        hist[i], valid[i] = h, v
    # exercise the general deque too: random valid patterns and positions
    rng = np.random.default_rng(7)
    for i in range(n // 2, n):
        valid[i] = rng.integers(0, 2, 8)
        valid[i, 7] = 1
        hist[i, :7] = pos[rng.integers(len(pos), size=7)]
    got = K.encode(hist, valid)
    for i in range(n):
        ref = C.full_state(hist[i], valid[i], hist[i, 7])
        assert np.array_equal(got[i].astype(np.float64), ref), i


@pytest.mark.parametrize("idx,depth", [(0, 5), (1, 4), (2, 5), (3, 4), (4, 4), (5, 4)])
def test_perft_on_device(K, idx, depth):
    from test_chess_oracle import PERFT
    fen, counts = PERFT[idx]
    assert K.perft(C.from_fen(fen), depth) == counts[depth - 1]


def test_perft_start_position_depth_6(K):
    """119,060,324 leaves: 5.4M positions expanded on the device."""
    assert K.perft(C.from_fen(), 6) == 119060324


def test_board_api_against_oracle(K):
    from custom_alphazero.chess.board import Board
    from custom_alphazero.chess.move import Move
    from custom_alphazero.chess.utils import get_all_possible_moves
    am = get_all_possible_moves()
    rng = np.random.default_rng(1)
    b = Board()
    ref = C.from_fen()
    assert [m.uci for m in b.moves] == [C.uci(m) for m in C.legal_moves(ref)]
    h, v = C.reference_history(ref, True)
    assert np.array_equal(b.full_state, C.full_state(h, v, ref))
    for ply in range(60):
        moves = b.moves
        if not moves or b.is_game_over():
            break
        assert np.array_equal(b.legal_moves_mask(am), C.legal_mask(ref, C.all_moves()).astype(bool))
        m = moves[rng.integers(len(moves))]
        child = b.play(m, on_copy=True, keep_same_player=True)
        ref = C.play_canonical(ref, m.code)
        h, v = C.reference_history(ref, False)
        assert np.array_equal(child.full_state, C.full_state(h, v, ref)), ply
        assert child.turn and np.array_equal(child.array, C.array(ref))
        b = child
    assert Move(uci="e2e4") in am and len(am) == 1880


def test_board_results_and_repetition(K):
    from custom_alphazero.chess.board import Board
    from custom_alphazero.chess.move import Move
    fool = Board("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR")
    for u in ("f2f3", "e7e5", "g2g4", "d8h4"):
        fool.push_uci(u)
    assert fool.is_checkmate() and fool.result() == "0-1" and fool.get_result() == 1
    with pytest.raises(ValueError):
        Board().push_uci("e2e5")
    # knights out and back twice: the start position a third time
    b = Board()
    seq = ["g1f3", "g8f6", "f3g1", "f6g8"] * 2
    for u in seq:
        b.play(Move(uci=u))
    assert b.is_repetition() and b.state[0, 0, 13] == 1
    assert b.full_state[0, 0, 7 * 14 + 13] == 1


def test_chess_abi_errors(K):
    from custom_alphazero import engine as az
    L = az.load_library()
    assert L.az_chess_legal(0, None, -1, None, None, None, None) == -1  # AZ_E_INVALID
    assert L.az_chess_perft(0, None, 3, None) < 0
    assert L.az_chess_legal(99, None, 0, None, None, None, None) == 0  # n == 0: no work


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_round1_perft_scheme_is_deterministic(mode):
    """tests/native/perft_repro.hip reconstructs the round-1 device perft
    (per-lane scratch move list generated twice per position, child offsets
    uploaded by a null-stream hipMemcpy (mode 0) or on the kernel's stream
    (mode 1) before a non-blocking-stream expand kernel): Kiwipete perft(4)
    exact on every run and both passes' lists identical at every position."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "_build", "perft_repro")
    assert os.path.exists(exe), "tests/native not built (__graft_entry__.build() builds it)"
    r = subprocess.run([exe, str(mode), "3"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 of 3 runs wrong, 0 count mismatches, 0 list mismatches" in r.stdout
