"""Batched chess board kernels (include/az_chess.h) over numpy arrays.

Every call runs on the GPU through libaz; there is no CPU fallback (a missing
libaz.so or no visible HIP device raises AzError).  Positions are numpy
records of POS_DTYPE, the az_chess_pos layout.
"""
import numpy as np

from custom_alphazero import engine as az
from custom_alphazero.config import ConfigChess

POS_DTYPE = np.dtype([
    ("pieces", "<u8", (6,)), ("occupied_co", "<u8", (2,)), ("castling_rights", "<u8"),
    ("ep_square", "<i2"), ("turn", "u1"), ("repetition", "u1"),
    ("halfmove_clock", "<u2"), ("fullmove_number", "<u2"),
])
assert POS_DTYPE.itemsize == 80

MAX_MOVES = 256      # AZ_CHESS_MAX_MOVES
ACTIONS = 1880       # AZ_CHESS_ACTIONS
HISTORY = 8          # AZ_CHESS_HISTORY
PLANES = 118         # AZ_CHESS_PLANES
OUTCOME_NAMES = {0: None, 1: "checkmate", 2: "insufficient_material", 3: "stalemate",
                 4: "seventyfive_moves"}


def _ptr(a):
    return az._ptr(a)


def _positions(pos):
    return np.ascontiguousarray(np.atleast_1d(pos), POS_DTYPE)


def all_moves():
    """get_all_possible_moves() as uint16 codes, in action order."""
    out = np.zeros(ACTIONS, np.uint16)
    n = az.load_library().az_chess_all_moves(_ptr(out), ACTIONS)
    if n < 0:
        az._check(n)
    return out[:n]


def legal(pos, device=None):
    """-> (moves [n][MAX_MOVES] u16, counts [n], mask [n][ACTIONS] bool, outcome [n])"""
    p = _positions(pos)
    n = len(p)
    moves = np.zeros((n, MAX_MOVES), np.uint16)
    counts = np.zeros(n, np.int32)
    mask = np.zeros((n, ACTIONS), np.uint8)
    outcome = np.zeros(n, np.int32)
    dev = ConfigChess.device if device is None else device
    az._check(az.load_library().az_chess_legal(int(dev), _ptr(p), n, _ptr(moves), _ptr(counts),
                                               _ptr(mask), _ptr(outcome)))
    return moves, counts, mask.astype(bool), outcome


def encode(hist, valid, device=None):
    """hist [n][8] positions oldest first, valid [n][8] -> state [n][8][8][118] f32"""
    h = np.ascontiguousarray(hist, POS_DTYPE).reshape(-1, HISTORY)
    v = np.ascontiguousarray(valid, np.uint8).reshape(-1, HISTORY)
    assert len(h) == len(v)
    out = np.zeros((len(h), 8, 8, PLANES), np.float32)
    dev = ConfigChess.device if device is None else device
    az._check(az.load_library().az_chess_encode(int(dev), _ptr(h), _ptr(v), len(h), _ptr(out)))
    return out


def play(pos, moves, keep_same_player=True, device=None):
    """Board.play on n positions (returns new records)"""
    p = _positions(pos).copy()
    m = np.ascontiguousarray(np.atleast_1d(moves), np.uint16)
    assert len(m) == len(p)
    dev = ConfigChess.device if device is None else device
    az._check(az.load_library().az_chess_play(int(dev), _ptr(p), _ptr(m), len(p),
                                              int(bool(keep_same_player))))
    return p


def perft(pos, depth, device=None):
    p = _positions(pos)[:1]
    out = np.zeros(1, np.uint64)
    dev = ConfigChess.device if device is None else device
    az._check(az.load_library().az_chess_perft(int(dev), _ptr(p), int(depth), _ptr(out)))
    return int(out[0])
