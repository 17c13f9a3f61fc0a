"""ctypes front-end of the C oracle (oracle/az_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  It is the checker
the GPU engine's outputs are compared against; its own parity is pinned by
tests/test_oracle.py against golden vectors produced by the real reference
(tests/golden/make_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

EVAL_SYNTH, EVAL_TABLE, EVAL_CALLBACK = 0, 1, 2


class GameOut(ctypes.Structure):
    _fields_ = [
        ("T", ctypes.c_int32), ("result", ctypes.c_int32), ("status", ctypes.c_int32),
        ("expansions", ctypes.c_int64), ("terminal_visits", ctypes.c_int64),
        ("nodes", ctypes.c_int64), ("max_depth", ctypes.c_int64),
    ]


EVAL_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int8),
                           ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float))

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.orc_pow_half.restype = ctypes.c_double
        L.orc_pow_half.argtypes = [ctypes.c_int64]
        L.orc_seed_uniform.restype = ctypes.c_double
        L.orc_seed_uniform.argtypes = [ctypes.c_uint32, ctypes.c_int]
        L.orc_choice.restype = ctypes.c_int
        L.orc_choice.argtypes = [P, ctypes.c_int, ctypes.c_double]
        L.orc_normalize_f32.restype = ctypes.c_int
        L.orc_normalize_f32.argtypes = [P, ctypes.c_int, P]
        L.orc_normalize_f64.restype = None
        L.orc_normalize_f64.argtypes = [P, ctypes.c_int, P]
        L.orc_board_replay.restype = ctypes.c_int
        L.orc_board_replay.argtypes = [ctypes.c_int] * 4 + [P, ctypes.c_int, P, P, P, P]
        L.orc_synth_probe.restype = None
        L.orc_synth_probe.argtypes = [ctypes.c_int] * 3 + [P, P, P]
        L.orc_table_new.restype = P
        L.orc_table_new.argtypes = [ctypes.c_int64, ctypes.c_int64, P, P, P]
        L.orc_table_free.restype = None
        L.orc_table_free.argtypes = [P]
        L.orc_table_misses.restype = ctypes.c_int64
        L.orc_table_misses.argtypes = [P]
        L.orc_play_game.restype = ctypes.c_int
        L.orc_set_noise.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double]
        L.orc_set_noise.restype = None
        L.orc_set_rng_skip.argtypes = [ctypes.c_int]
        L.orc_set_rng_skip.restype = None
        L.orc_dirichlet_draws.argtypes = [ctypes.c_uint32, ctypes.c_double, ctypes.c_int, ctypes.c_int, P]
        L.orc_dirichlet_draws.restype = None
        L.orc_play_game.argtypes = (
            [ctypes.c_int] * 5 + [ctypes.c_uint32, ctypes.c_int, P, EVAL_CB, P]
            + [P] * 10 + [ctypes.POINTER(GameOut)])
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def action_space(width, height, gravity):
    return width if gravity else width * height


def pow_half(n):
    return lib().orc_pow_half(int(n))


def seed_uniform(seed, k):
    return lib().orc_seed_uniform(int(seed), int(k))


def choice(p, u):
    p = np.ascontiguousarray(p, np.float64)
    return lib().orc_choice(_ptr(p), len(p), float(u))


def normalize_f32(p):
    p = np.ascontiguousarray(p, np.float32)
    out = np.zeros(len(p), np.float64)
    uniform = lib().orc_normalize_f32(_ptr(p), len(p), _ptr(out))
    return out, bool(uniform)


def normalize_f64(p):
    p = np.ascontiguousarray(p, np.float64)
    out = np.zeros(len(p), np.float64)
    lib().orc_normalize_f64(_ptr(p), len(p), _ptr(out))
    return out


def board_replay(height, width, n, gravity, actions):
    actions = np.ascontiguousarray(actions, np.int32)
    k = len(actions)
    A = action_space(width, height, gravity)
    boards = np.zeros((k, height, width), np.int8)
    status = np.zeros(k, np.int32)
    mask = np.zeros((k, A), np.uint8)
    moves = np.zeros((k, A), np.int32)
    rc = lib().orc_board_replay(height, width, n, int(gravity), _ptr(actions), k, _ptr(boards),
                                _ptr(status), _ptr(mask), _ptr(moves))
    if rc:
        raise ValueError("illegal action in replay")
    return boards, status, mask.astype(bool), moves


def synth_probe(board, gravity):
    board = np.ascontiguousarray(board, np.int8)
    height, width = board.shape
    A = action_space(width, height, gravity)
    probs = np.zeros(A, np.float32)
    value = np.zeros(1, np.float32)
    lib().orc_synth_probe(height, width, int(gravity), _ptr(board), _ptr(probs), _ptr(value))
    return probs, float(value[0])


class EvalTable:
    """(board masks -> probs, value) replay table; keys are [n, 4] uint64
    (own_lo, own_hi, opp_lo, opp_hi)."""

    def __init__(self, keys, probs, values):
        keys = np.ascontiguousarray(keys, np.uint64).reshape(-1, 4)
        probs = np.ascontiguousarray(probs, np.float32).reshape(len(keys), -1)
        values = np.ascontiguousarray(values, np.float32).reshape(-1)
        self._keep = (keys, probs, values)
        self.handle = lib().orc_table_new(len(keys), probs.shape[1], _ptr(keys), _ptr(probs),
                                          _ptr(values))

    def misses(self):
        return lib().orc_table_misses(self.handle)

    def __del__(self):
        if getattr(self, "handle", None):
            lib().orc_table_free(self.handle)
            self.handle = None


def dirichlet_draws(seed, alpha, k, n):
    """n draws of np.random.dirichlet(alpha * ones(k)) from a legacy stream
    seeded `seed` (the C restatement, libm log/pow as numpy calls them)."""
    out = np.zeros((n, k), np.float64)
    lib().orc_dirichlet_draws(int(seed) & 0xFFFFFFFF, float(alpha), int(k), int(n), _ptr(out))
    return out


def play_game(height, width, n, gravity, sims, seed, evaluator="synth", table=None,
              callback=None, noise=None, rng_skip=None):
    """One reference self-play game (self_play.py:37-82) on the C oracle.

    evaluator: "synth" (oracle/synth.py), "table" (EvalTable), or "callback"
    (python callable board[H,W] int8 -> (probs[A] f32, value f32)).
    noise: None, or (alpha, ratio) -- ConfigMCTS.enable_dirichlet_noise with
    dirichlet_noise_value / dirichlet_noise_ratio (mcts.py:70-85).
    rng_skip: MT19937 words discarded after seeding; None = the reference
    play_game's model construction, np.random.rand(1, H, W, 4) (2 H W 4).
    """
    lib().orc_set_noise(int(noise is not None), *(noise if noise is not None else (0.03, 0.25)))
    lib().orc_set_rng_skip(-1 if rng_skip is None else int(rng_skip))
    try:
        return _play_game(height, width, n, gravity, sims, seed, evaluator, table, callback)
    finally:
        lib().orc_set_noise(0, 0.03, 0.25)
        lib().orc_set_rng_skip(-1)


def _play_game(height, width, n, gravity, sims, seed, evaluator, table, callback):
    A = action_space(width, height, gravity)
    T = height * width
    o = {
        "moves": np.zeros(T, np.int32), "greedy": np.zeros(T, np.uint8),
        "n_edges": np.zeros(T, np.int32), "edge_action": np.zeros((T, A), np.int32),
        "edge_prior": np.zeros((T, A), np.float64), "edge_n": np.zeros((T, A), np.int64),
        "edge_w": np.zeros((T, A), np.float64), "policy": np.zeros((T, A), np.float64),
        "boards": np.zeros((T, height, width), np.int8), "rewards": np.zeros(T, np.int64),
    }
    out = GameOut()
    kind = {"synth": EVAL_SYNTH, "table": EVAL_TABLE, "callback": EVAL_CALLBACK}[evaluator]
    cb = EVAL_CB(0)
    if kind == EVAL_CALLBACK:
        def _cb(_ctx, bptr, pptr, vptr):
            b = np.ctypeslib.as_array(bptr, shape=(height, width)).copy()
            p, v = callback(b)
            p = np.asarray(p, np.float32)
            for i in range(A):
                pptr[i] = float(p[i])
            vptr[0] = float(np.float32(v))
            return 0
        cb = EVAL_CB(_cb)
    rc = lib().orc_play_game(
        height, width, n, int(gravity), sims, int(seed) & 0xFFFFFFFF, kind,
        table.handle if table is not None else None, cb, None,
        _ptr(o["moves"]), _ptr(o["greedy"]), _ptr(o["n_edges"]), _ptr(o["edge_action"]),
        _ptr(o["edge_prior"]), _ptr(o["edge_n"]), _ptr(o["edge_w"]), _ptr(o["policy"]),
        _ptr(o["boards"]), _ptr(o["rewards"]), ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(f"oracle play_game failed rc={rc}")
    t = out.T
    res = {k: v[:t] for k, v in o.items()}
    res["greedy"] = res["greedy"].astype(bool)
    res.update(T=t, result=out.result, expansions=out.expansions,
               terminal_visits=out.terminal_visits, nodes=out.nodes, max_depth=out.max_depth)
    return res


def full_state(boards):
    """Board.full_state (connect_n/board.py:91-98) for canonical boards [..., H, W]:
    channels [empty, +1, -1, turn=1]."""
    b = np.asarray(boards)
    s = np.zeros(b.shape + (4,), np.float32)
    s[..., 0] = b == 0
    s[..., 1] = b == 1
    s[..., 2] = b == -1
    s[..., 3] = 1.0
    return s


def board_keys(boards):
    """[n, H, W] canonical boards -> [n, 4] uint64 (own_lo, own_hi, opp_lo, opp_hi)."""
    b = np.asarray(boards).reshape(len(boards), -1)
    keys = np.zeros((len(b), 4), np.uint64)
    for half in range(2):
        cells = b[:, 64 * half: 64 * (half + 1)]
        if cells.shape[1] == 0:
            continue
        bits = (np.uint64(1) << np.arange(cells.shape[1], dtype=np.uint64))
        keys[:, half] = ((cells == 1) * bits).sum(axis=1, dtype=np.uint64)
        keys[:, 2 + half] = ((cells == -1) * bits).sum(axis=1, dtype=np.uint64)
    return keys
