"""ctypes front-end of the chess oracle (oracle/chess_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/ and __graft_entry__.smoke(),
never by the product package.  It checks the HIP chess kernels
(csrc/az_chess.hip).  Its legal-move sets are pinned by published perft
counts (tests/test_chess_oracle.py); generation order, history planes and
outcome rules restate python-chess 1.9.4 and are "parity unpinned" (python-chess
is absent here, the reference holds no chess fixture).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libchess_oracle.so")

# az_chess_pos (include/az_chess.h) as a numpy record: 80 bytes
POS_DTYPE = np.dtype([
    ("pieces", "<u8", (6,)), ("occupied_co", "<u8", (2,)), ("castling_rights", "<u8"),
    ("ep_square", "<i2"), ("turn", "u1"), ("repetition", "u1"),
    ("halfmove_clock", "<u2"), ("fullmove_number", "<u2"),
])
assert POS_DTYPE.itemsize == 80

START_FEN = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
PIECE_TYPES = {0: "", 2: "n", 3: "b", 4: "r", 5: "q"}
OUTCOMES = {0: None, 1: "checkmate", 2: "insufficient_material", 3: "stalemate",
            4: "seventyfive_moves"}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.orc_chess_pos_size.restype = ctypes.c_int
        assert L.orc_chess_pos_size() == POS_DTYPE.itemsize
        L.orc_chess_from_fen.argtypes = [ctypes.c_char_p, P]
        L.orc_chess_legal.argtypes = [P, P]
        L.orc_chess_legal.restype = ctypes.c_int
        L.orc_chess_push.argtypes = [P, ctypes.c_uint16]
        L.orc_chess_mirror.argtypes = [P]
        L.orc_chess_play_canonical.argtypes = [P, ctypes.c_uint16]
        L.orc_chess_outcome.argtypes = [P]
        L.orc_chess_outcome.restype = ctypes.c_int
        L.orc_chess_perft.argtypes = [P, ctypes.c_int]
        L.orc_chess_perft.restype = ctypes.c_uint64
        L.orc_chess_array.argtypes = [P, P]
        L.orc_chess_full_state.argtypes = [P, P, P, P]
        L.orc_chess_all_moves.argtypes = [P]
        L.orc_chess_all_moves.restype = ctypes.c_int
        L.orc_chess_legal_mask.argtypes = [P, P, ctypes.c_int, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def from_fen(fen=START_FEN):
    p = np.zeros(1, POS_DTYPE)
    if lib().orc_chess_from_fen(fen.encode(), _p(p)) != 0:
        raise ValueError(fen)
    return p[0]


def _one(pos):
    return np.array([pos], POS_DTYPE)


def legal_moves(pos):
    out = np.zeros(256, np.uint16)
    n = lib().orc_chess_legal(_p(_one(pos)), _p(out))
    return out[:n].copy()


def push(pos, move):
    p = _one(pos)
    lib().orc_chess_push(_p(p), int(move))
    return p[0]


def mirror(pos):
    p = _one(pos)
    lib().orc_chess_mirror(_p(p))
    return p[0]


def play_canonical(pos, move):
    """Board.play(move, keep_same_player=True) (chess/board.py:162-173)."""
    p = _one(pos)
    lib().orc_chess_play_canonical(_p(p), int(move))
    return p[0]


def outcome(pos):
    return lib().orc_chess_outcome(_p(_one(pos)))


def perft(pos, depth):
    return int(lib().orc_chess_perft(_p(_one(pos)), depth))


def array(pos):
    out = np.zeros(64, np.int8)
    lib().orc_chess_array(_p(_one(pos)), _p(out))
    return out.reshape(8, 8)


def full_state(hist, valid, cur):
    """hist: 8 positions oldest first; valid: 8 flags; -> float64 [8][8][118]."""
    h = np.array(hist, POS_DTYPE)
    v = np.ascontiguousarray(valid, np.uint8)
    out = np.zeros((8, 8, 118), np.float64)
    lib().orc_chess_full_state(_p(h), _p(v), _p(_one(cur)), _p(out))
    return out


def reference_history(pos, is_root):
    """The history deque the reference's boards carry in MCTS use.  The root
    node's board is a deepcopy (mcts.py:96, 107), and python-chess's copy()
    re-runs the subclass __init__ (start position), so it holds [0 x 7,
    start-position state] whatever the position (for a game's first Board(),
    the start position itself); every board made by play() holds [0 x 6,
    start-position state, state]."""
    start = from_fen(START_FEN)
    hist = [start] * 8
    valid = [0] * 8
    valid[7] = 1
    if not is_root:
        hist[7] = pos
        hist[6], valid[6] = start, 1
    return hist, valid


def all_moves():
    out = np.zeros(4096, np.uint16)
    n = lib().orc_chess_all_moves(_p(out))
    return out[:n].copy()


def legal_mask(pos, all_mv):
    all_mv = np.ascontiguousarray(all_mv, np.uint16)
    mask = np.zeros(len(all_mv), np.uint8)
    lib().orc_chess_legal_mask(_p(_one(pos)), _p(all_mv), len(all_mv), _p(mask))
    return mask


def uci(move):
    f, t, pr = int(move) & 63, (int(move) >> 6) & 63, int(move) >> 12
    sq = lambda s: "abcdefgh"[s & 7] + str((s >> 3) + 1)
    return sq(f) + sq(t) + PIECE_TYPES[pr]


def random_positions(n, seed, max_plies=200, canonical=True):
    """Positions reached by seeded random playouts from the start position
    (canonical = Board.play(keep_same_player=True) after every move, as in
    MCTS).  Returns (positions, is_root flags)."""
    rng = np.random.default_rng(seed)
    out, roots = [], []
    pos = from_fen()
    is_root = True
    ply = 0
    while len(out) < n:
        out.append(pos)
        roots.append(is_root)
        mv = legal_moves(pos)
        if len(mv) == 0 or outcome(pos) != 0 or ply >= max_plies:
            pos, is_root, ply = from_fen(), True, 0
            continue
        m = mv[rng.integers(len(mv))]
        pos = play_canonical(pos, m) if canonical else push(pos, m)
        is_root = False
        ply += 1
    return np.array(out, POS_DTYPE), np.array(roots, bool)


class ChessGameOut(ctypes.Structure):
    _fields_ = [("T", ctypes.c_int32), ("result", ctypes.c_int32), ("termination", ctypes.c_int32),
                ("expansions", ctypes.c_int64), ("terminal_visits", ctypes.c_int64)]


CHESS_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                            ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float))


def play_game(sims, seed, max_plies, greedy_ply=8, c_puct=1.5, callback=None):
    """One chess self-play game on the oracle.  callback(pos, initial) ->
    (probs f32[1880], value) replaces the synthetic evaluator (network replay)."""
    L = lib()
    fn = L.orc_chess_play_game
    fn.restype = ctypes.c_int
    P = ctypes.c_void_p
    fn.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                   ctypes.c_int, CHESS_CB, P, P, P, P, P, P, P, ctypes.POINTER(ChessGameOut)]
    positions = np.zeros(max_plies, POS_DTYPE)
    moves = np.zeros(max_plies, np.uint16)
    pol_n = np.zeros(max_plies, np.int32)
    pol_a = np.zeros((max_plies, 256), np.int16)
    pol_p = np.zeros((max_plies, 256), np.float64)
    visits = np.zeros((max_plies, 256), np.int64)
    out = ChessGameOut()
    err = []

    def _cb(ctx, pos_ptr, initial, probs_ptr, value_ptr):
        try:
            raw = ctypes.string_at(pos_ptr, POS_DTYPE.itemsize)
            pos = np.frombuffer(raw, POS_DTYPE)[0]
            p, v = callback(pos, int(initial))
            p = np.ascontiguousarray(p, np.float32)
            ctypes.memmove(probs_ptr, p.ctypes.data, 4 * 1880)
            value_ptr[0] = float(v)
            return 0
        except Exception as e:  # pragma: no cover - surfaced below
            err.append(e)
            return 1

    cb = CHESS_CB(_cb) if callback is not None else CHESS_CB()
    rc = fn(sims, seed & 0xFFFFFFFF, max_plies, greedy_ply, c_puct, 1 if callback else 0, cb, None,
            _p(positions), _p(moves), _p(pol_n), _p(pol_a), _p(pol_p), _p(visits), ctypes.byref(out))
    if err:
        raise err[0]
    assert rc == 0, "oracle chess game failed"
    T = out.T
    return dict(T=T, result=out.result, termination=out.termination, expansions=out.expansions,
                terminal_visits=out.terminal_visits, positions=positions[:T], moves=moves[:T],
                policy_n=pol_n[:T], policy_actions=pol_a[:T], policy_probs=pol_p[:T],
                root_visits=visits[:T])


def synth(pos, initial):
    L = lib()
    L.orc_chess_synth.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    probs = np.zeros(1880, np.float32)
    v = np.zeros(1, np.float32)
    L.orc_chess_synth(_p(_one(pos)), int(initial), _p(probs), _p(v))
    return probs, float(v[0])


class Tree:
    """One MCTS object (mcts.py:86-222) on a chess root, on the oracle
    (orc_chess_tree_*): search(n), play(u, greedy, deterministic), root()."""

    def __init__(self, root, c_puct=1.5, callback=None):
        L = lib()
        P = ctypes.c_void_p
        L.orc_chess_tree_new.restype = P
        L.orc_chess_tree_new.argtypes = [P, ctypes.c_double, ctypes.c_int, CHESS_CB, P]
        L.orc_chess_tree_search.argtypes = [P, ctypes.c_int]
        L.orc_chess_tree_play.argtypes = [P, ctypes.c_double, ctypes.c_int, ctypes.c_int, P, P, P, P]
        L.orc_chess_tree_play.restype = ctypes.c_int
        L.orc_chess_tree_root.argtypes = [P, P, P, P, P, P]
        L.orc_chess_tree_root.restype = ctypes.c_int
        L.orc_chess_tree_expansions.argtypes = [P]
        L.orc_chess_tree_expansions.restype = ctypes.c_int64
        L.orc_chess_tree_error.argtypes = [P]
        L.orc_chess_tree_error.restype = ctypes.c_int
        L.orc_chess_tree_free.argtypes = [P]
        self._L, self._err, self._callback = L, [], callback

        def _cb(ctx, pos_ptr, initial, probs_ptr, value_ptr):
            try:
                pos = np.frombuffer(ctypes.string_at(pos_ptr, POS_DTYPE.itemsize), POS_DTYPE)[0]
                p, v = callback(pos, int(initial))
                p = np.ascontiguousarray(p, np.float32)
                ctypes.memmove(probs_ptr, p.ctypes.data, 4 * 1880)
                value_ptr[0] = float(v)
                return 0
            except Exception as e:  # pragma: no cover - surfaced by _check
                self._err.append(e)
                return 1

        self._cb = CHESS_CB(_cb) if callback is not None else CHESS_CB()
        self._root = _one(root)
        self._h = L.orc_chess_tree_new(_p(self._root), c_puct, 1 if callback else 0, self._cb, None)

    def _check(self):
        if self._err:
            raise self._err[0]
        assert self._L.orc_chess_tree_error(self._h) == 0

    def search(self, n):
        self._L.orc_chess_tree_search(self._h, int(n))
        self._check()

    def play(self, u=0.0, greedy=False, deterministic=False):
        mv = np.zeros(1, np.uint16)
        n = np.zeros(1, np.int32)
        pa = np.zeros(256, np.int16)
        pp = np.zeros(256, np.float64)
        oc = self._L.orc_chess_tree_play(self._h, float(u), int(greedy), int(deterministic), _p(mv), _p(n),
                                         _p(pa), _p(pp))
        if oc < 0:
            raise RuntimeError("play() before search")
        k = int(n[0])
        return int(mv[0]), oc, pa[:k].copy(), pp[:k].copy()

    def root(self):
        mv = np.zeros(256, np.uint16)
        prior = np.zeros(256, np.float64)
        N = np.zeros(256, np.int64)
        W = np.zeros(256, np.float64)
        cn = np.zeros(256, np.int32)
        k = self._L.orc_chess_tree_root(self._h, _p(mv), _p(prior), _p(N), _p(W), _p(cn))
        return dict(moves=mv[:k], prior=prior[:k], n=N[:k], w=W[:k], child_n=cn[:k])

    @property
    def expansions(self):
        return int(self._L.orc_chess_tree_expansions(self._h))

    def close(self):
        if getattr(self, "_h", None):
            self._L.orc_chess_tree_free(self._h)
            self._h = None

    def __del__(self):
        self.close()
