"""ctypes binding of libaz (include/az.h): the only way this package computes.

There is deliberately no CPU fallback: if ``_lib/libaz.so`` is missing or no
HIP device is visible, every entry point raises.  The reference's evaluator,
tree and worker seams all land here.
"""
import ctypes
import os

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libaz.so")

EVAL_NETWORK = 0
EVAL_SYNTHETIC = 1
EVAL_HOST = 2  # include/az.h AZ_EVAL_HOST: a Python callable (Engine.set_host_evaluator)
CONV_F16X2 = 0  # include/az.h AZ_CONV_F16X2 (default)
CONV_DIRECT = 1
CONV_F16X2_LAYERS = 2  # AZ_CONV_F16X2_LAYERS: the same arithmetic one layer per launch (A/B runs)


class AzError(RuntimeError):
    pass


class Config(ctypes.Structure):
    _fields_ = [
        ("board_height", ctypes.c_int32), ("board_width", ctypes.c_int32),
        ("n", ctypes.c_int32), ("gravity", ctypes.c_int32),
        ("mcts_iterations", ctypes.c_int32), ("index_move_greedy", ctypes.c_int32),
        ("exploration_constant", ctypes.c_double), ("slots", ctypes.c_int32),
        ("evaluator", ctypes.c_int32), ("filters", ctypes.c_int32), ("depth", ctypes.c_int32),
        ("value_hidden", ctypes.c_int32), ("bn_epsilon", ctypes.c_double),
        ("arena_edges", ctypes.c_int64), ("max_tree_visits", ctypes.c_int64),
        ("cache_log2", ctypes.c_int32), ("conv_algo", ctypes.c_int32),
        ("lanes", ctypes.c_int32), ("compact", ctypes.c_int32),
        ("tower_natural_order", ctypes.c_int32), ("dirichlet_noise", ctypes.c_int32),
        ("dirichlet_alpha", ctypes.c_double), ("dirichlet_ratio", ctypes.c_double),
        ("rng_skip", ctypes.c_int32), ("reserved", ctypes.c_int32 * 1),
    ]


class ChessConfig(ctypes.Structure):
    """az_chess_config (include/az_chess.h)."""
    _fields_ = [
        ("mcts_iterations", ctypes.c_int32), ("index_move_greedy", ctypes.c_int32),
        ("exploration_constant", ctypes.c_double), ("slots", ctypes.c_int32),
        ("evaluator", ctypes.c_int32), ("filters", ctypes.c_int32), ("depth", ctypes.c_int32),
        ("value_hidden", ctypes.c_int32), ("max_plies", ctypes.c_int32),
        ("bn_epsilon", ctypes.c_double), ("arena_edges", ctypes.c_int64),
        ("conv_algo", ctypes.c_int32), ("lanes", ctypes.c_int32), ("cache_log2", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 5),
    ]


class Tensor(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("numel", ctypes.c_int64),
                ("on_device", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [
        ("expansions", ctypes.c_int64), ("terminal_visits", ctypes.c_int64),
        ("games_done", ctypes.c_int64), ("simulations", ctypes.c_int64),
        ("plies", ctypes.c_int64), ("active_slots", ctypes.c_int64), ("errors", ctypes.c_int64),
        ("conv_launches", ctypes.c_int64), ("conv_ms", ctypes.c_double),
        ("cache_hits", ctypes.c_int64), ("evaluations", ctypes.c_int64),
        ("conv_busy_ms", ctypes.c_double), ("tree_launches", ctypes.c_int64), ("tree_ms", ctypes.c_double),
        ("path_edges", ctypes.c_int64), ("cache_inserts", ctypes.c_int64),
        ("cache_generation", ctypes.c_int64), ("cache_gen_size", ctypes.c_int64),
        ("cache_capacity", ctypes.c_int64), ("games_drained", ctypes.c_int64),
        ("max_retained", ctypes.c_int64), ("cache_entries", ctypes.c_int64),
        ("arena_edges", ctypes.c_int64), ("issued_flop_per_board", ctypes.c_double),
        ("arena_pool_edges", ctypes.c_int64), ("arena_pool_high", ctypes.c_int64),
        ("issued_flop_per_board_small", ctypes.c_double), ("tower_small_max_boards", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


# az_eval_fn (include/az.h): (user, x [n][H][W][4], n, probs [n][A], values [n]) -> 0 / nonzero
EVAL_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int32,
                           ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float))


def _as_numpy(t):
    """A model output (numpy, torch or TF tensor, list) as a numpy array."""
    if hasattr(t, "detach"):
        t = t.detach().cpu()
    if hasattr(t, "numpy"):
        t = t.numpy()
    return np.asarray(t)


EXPORTED = (
    "az_abi_version", "az_last_error", "az_build_id", "az_build_flags", "az_engine_create", "az_engine_destroy",
    "az_engine_lanes",
    "az_engine_set_weights", "az_encode", "az_forward", "az_selfplay_begin", "az_selfplay_step",
    "az_selfplay_run", "az_selfplay_results", "az_selfplay_drain", "az_tree_reset", "az_tree_release", "az_tree_search", "az_tree_search_noise", "az_tree_play",
    "az_tree_info", "az_tree_export", "az_stats_get", "az_timer_enable", "az_pow_table",
    "az_cache_clear", "az_cache_enable", "az_engine_set_evaluator",
    # include/az_chess.h
    "az_chess_all_moves", "az_chess_legal", "az_chess_encode", "az_chess_play", "az_chess_perft",
    "az_chess_engine_create", "az_chess_engine_destroy", "az_chess_engine_set_weights",
    "az_chess_forward", "az_chess_selfplay_begin", "az_chess_selfplay_step", "az_chess_selfplay_run",
    "az_chess_selfplay_results", "az_chess_selfplay_drain", "az_chess_stats", "az_chess_timer_enable",
    "az_chess_tree_reset",
    "az_chess_tree_release", "az_chess_tree_search", "az_chess_tree_play", "az_chess_tree_info",
    "az_chess_tree_export",
)

_lib = None


def load_library():
    """Load libaz.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("AZ_LIB_PATH", LIB_PATH)  # A/B builds (profiles/); default in-tree lib
    if not os.path.exists(path):
        raise AzError(f"libaz.so not built at {path}; run __graft_entry__.build()")
    # One HIP runtime per process: torch's wheel bundles its own libamdhip64 /
    # libhsa-runtime64 with the same SONAMEs as /opt/rocm's.  Loading torch
    # first makes libaz bind to that already-loaded runtime (SONAME match);
    # the reverse order leaves two runtimes and torch then sees no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        "az_abi_version": (ctypes.c_int, []),
        "az_last_error": (ctypes.c_char_p, []),
        "az_build_id": (ctypes.c_char_p, []),
        "az_build_flags": (ctypes.c_char_p, []),
        "az_engine_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(Config), ctypes.POINTER(P)]),
        "az_engine_destroy": (ctypes.c_int, [P]),
        "az_engine_lanes": (ctypes.c_int, [P]),
        "az_engine_set_weights": (ctypes.c_int, [P, ctypes.POINTER(Tensor), ctypes.c_int]),
        "az_encode": (ctypes.c_int, [P, P, ctypes.c_int, P, P]),
        "az_forward": (ctypes.c_int, [P, P, ctypes.c_int, P, P]),
        "az_selfplay_begin": (ctypes.c_int, [P, I64, I64, ctypes.c_uint32]),
        "az_selfplay_step": (ctypes.c_int, [P, ctypes.c_int, ctypes.POINTER(Stats)]),
        "az_selfplay_run": (ctypes.c_int, [P, I64, I64, ctypes.c_uint32, ctypes.POINTER(Stats)]),
        "az_selfplay_results": (ctypes.c_int, [P, P, P, P, P, P, P]),
        "az_selfplay_drain": (ctypes.c_int, [P, I64, P, P, P, P, P, P, P, P]),
        "az_tree_reset": (ctypes.c_int, [P, ctypes.c_int, P, P]),
        "az_tree_release": (ctypes.c_int, [P, ctypes.c_int, P]),
        "az_tree_search": (ctypes.c_int, [P, ctypes.c_int]),
        "az_tree_search_noise": (ctypes.c_int, [P, ctypes.c_int, P, ctypes.c_int]),
        "az_tree_play": (ctypes.c_int, [P, P, ctypes.c_int, ctypes.c_int, P, P, P]),
        "az_tree_info": (ctypes.c_int, [P, ctypes.c_int, P, P]),
        "az_tree_export": (ctypes.c_int, [P, ctypes.c_int, P, P, P, P, P, P, P]),
        "az_stats_get": (ctypes.c_int, [P, ctypes.POINTER(Stats)]),
        "az_timer_enable": (ctypes.c_int, [P, ctypes.c_int]),
        "az_pow_table": (ctypes.c_int, [P, P, I64]),
        "az_cache_clear": (ctypes.c_int, [P]),
        "az_cache_enable": (ctypes.c_int, [P, ctypes.c_int]),
        "az_engine_set_evaluator": (ctypes.c_int, [P, EVAL_FN, P]),
        "az_chess_all_moves": (ctypes.c_int, [P, ctypes.c_int]),
        "az_chess_legal": (ctypes.c_int, [ctypes.c_int, P, ctypes.c_int, P, P, P, P]),
        "az_chess_encode": (ctypes.c_int, [ctypes.c_int, P, P, ctypes.c_int, P]),
        "az_chess_play": (ctypes.c_int, [ctypes.c_int, P, P, ctypes.c_int, ctypes.c_int]),
        "az_chess_perft": (ctypes.c_int, [ctypes.c_int, P, ctypes.c_int, P]),
        "az_chess_engine_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ChessConfig),
                                                  ctypes.POINTER(P)]),
        "az_chess_engine_destroy": (ctypes.c_int, [P]),
        "az_chess_engine_set_weights": (ctypes.c_int, [P, ctypes.POINTER(Tensor), ctypes.c_int]),
        "az_chess_forward": (ctypes.c_int, [P, P, ctypes.c_int, P, P]),
        "az_chess_selfplay_begin": (ctypes.c_int, [P, I64, I64, ctypes.c_uint32]),
        "az_chess_selfplay_step": (ctypes.c_int, [P, ctypes.c_int, ctypes.POINTER(Stats)]),
        "az_chess_selfplay_run": (ctypes.c_int, [P, I64, I64, ctypes.c_uint32, ctypes.POINTER(Stats)]),
        "az_chess_selfplay_results": (ctypes.c_int, [P] + [P] * 9),
        "az_chess_selfplay_drain": (ctypes.c_int, [P, I64, P] + [P] * 10),
        "az_chess_stats": (ctypes.c_int, [P, ctypes.POINTER(Stats)]),
        "az_chess_timer_enable": (ctypes.c_int, [P, ctypes.c_int]),
        "az_chess_tree_reset": (ctypes.c_int, [P, ctypes.c_int, P, P]),
        "az_chess_tree_release": (ctypes.c_int, [P, ctypes.c_int, P]),
        "az_chess_tree_search": (ctypes.c_int, [P, ctypes.c_int]),
        "az_chess_tree_play": (ctypes.c_int, [P, P, ctypes.c_int, ctypes.c_int, P, P, P, P, P]),
        "az_chess_tree_info": (ctypes.c_int, [P, ctypes.c_int, P, P]),
        "az_chess_tree_export": (ctypes.c_int, [P, ctypes.c_int, P, P, P, P, P, P, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _ = I32
    _lib = L
    return L


def build_id():
    """(source hash, extra compile flags) of the loaded libaz (az_build_id /
    az_build_flags): profiles record the hash, bench.py matches it."""
    L = load_library()
    return L.az_build_id().decode(), L.az_build_flags().decode()


def _check(rc):
    if rc != 0:
        msg = load_library().az_last_error().decode("utf-8", "replace")
        raise AzError(f"libaz error {rc}: {msg}")


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def tensor_array(named):
    """(name, numpy array or torch tensor) pairs -> az_tensor array; torch
    CUDA tensors are passed as device pointers (the engine copies them)."""
    keep, items = [], []
    for name, t in named:
        on_dev = 0
        if hasattr(t, "is_cuda"):
            t = t.detach().float().contiguous()
            on_dev = int(t.is_cuda)
            if not on_dev:
                t = t.numpy()
        if on_dev:
            ptr, numel = t.data_ptr(), t.numel()
        else:
            t = np.ascontiguousarray(t, np.float32)
            ptr, numel = t.ctypes.data, t.size
        keep.append(t)
        items.append(Tensor(name.encode(), ptr, numel, on_dev, 0))
    arr = (Tensor * len(items))(*items)
    if any(i.on_device for i in items):
        import torch
        torch.cuda.synchronize()
    return arr, len(items), keep


class Engine:
    """One libaz engine: one device, one HIP stream, `slots` concurrent trees."""

    def __init__(self, height=6, width=7, n=4, gravity=True, mcts_iterations=100, slots=1,
                 evaluator=EVAL_NETWORK, index_move_greedy=8, exploration_constant=1.5,
                 filters=128, depth=4, value_hidden=256, bn_epsilon=1e-3, arena_edges=0,
                 max_tree_visits=0, device=0, cache_log2=0, conv_algo=CONV_F16X2,
                 lanes=0, compact=False, tower_natural_order=False, dirichlet_noise=False,
                 dirichlet_alpha=0.03, dirichlet_ratio=0.25, rng_skip=None):
        """compact=True reclaims the subtrees a self-play game has left after
        every move (az_config.compact; arena_edges is then per half); keep it
        off for the tree API (az_tree_*), whose views need the whole tree.
        dirichlet_noise: ConfigMCTS.enable_dirichlet_noise (root noise,
        reference mcts.py:70-85) with dirichlet_alpha / dirichlet_ratio.
        rng_skip: MT19937 words a self-play game's stream discards after
        seeding; None = the reference play_game's model construction
        (np.random.rand(1, H, W, 4): 2 H W 4 words), so game g of a batch is
        the reference's play_game under np.random.seed(base_seed + g)."""
        L = load_library()
        self.height, self.width, self.n, self.gravity = height, width, n, bool(gravity)
        self.action_space = width if gravity else width * height
        self.slots = slots
        self.mcts_iterations = mcts_iterations
        cfg = Config(board_height=height, board_width=width, n=n, gravity=int(bool(gravity)),
                     mcts_iterations=mcts_iterations, index_move_greedy=index_move_greedy,
                     exploration_constant=exploration_constant, slots=slots, evaluator=evaluator,
                     filters=filters, depth=depth, value_hidden=value_hidden,
                     bn_epsilon=bn_epsilon, arena_edges=arena_edges,
                     max_tree_visits=max_tree_visits, cache_log2=cache_log2, conv_algo=conv_algo,
                     lanes=lanes, compact=int(bool(compact)),
                     tower_natural_order=int(bool(tower_natural_order)),
                     dirichlet_noise=int(bool(dirichlet_noise)), dirichlet_alpha=float(dirichlet_alpha),
                     dirichlet_ratio=float(dirichlet_ratio),
                     rng_skip=2 * height * width * 4 if rng_skip is None else int(rng_skip))
        handle = ctypes.c_void_p()
        _check(L.az_engine_create(int(device), ctypes.byref(cfg), ctypes.byref(handle)))
        self._h = handle
        self._L = L
        self._n_games = 0
        self._host_fn = None     # the EVAL_FN object (kept alive while the engine may call it)
        self._host_error = None  # an exception the host evaluator raised inside a search

    @property
    def lanes(self):
        """The slot groups (streams) the engine runs (az_engine_lanes)."""
        return int(self._L.az_engine_lanes(self._h))

    def close(self):
        if getattr(self, "_h", None):
            self._L.az_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter teardown
            pass

    # ------------------------------------------------------------- weights
    def set_weights(self, named):
        """named: iterable of (name, array-like or torch tensor)."""
        arr, n, _keep = tensor_array(named)
        _check(self._L.az_engine_set_weights(self._h, arr, n))

    def set_host_evaluator(self, fn):
        """EVAL_HOST engines: fn(x) with x [n, H, W, 4] float32 full_state planes
        returns (probs [n, A], values [n] or [n, 1]) -- the reference's
        self.model(x) call (mcts.py:130-137), here once per simulation over
        every leaf that needs an evaluation.  Outputs may be numpy arrays or
        torch / TF tensors.  An exception inside fn ends the search and is
        re-raised by the call that ran it."""
        H, W, A = self.height, self.width, self.action_space

        def cb(_user, xp, n, pp, vp):
            try:
                x = np.ctypeslib.as_array(xp, shape=(n, H, W, 4)).copy()
                p, v = fn(x)
                p = _as_numpy(p).astype(np.float32, copy=False).reshape(n, A)
                v = _as_numpy(v).astype(np.float32, copy=False).reshape(n)
                np.ctypeslib.as_array(pp, shape=(n, A))[:] = p
                np.ctypeslib.as_array(vp, shape=(n,))[:] = v
                return 0
            except BaseException as ex:  # noqa: BLE001 - handed back to the caller below
                self._host_error = ex
                return 1

        self._host_fn = EVAL_FN(cb)
        _check(self._L.az_engine_set_evaluator(self._h, self._host_fn, None))

    def _search_call(self, rc):
        """_check for calls that can run the host evaluator: its exception first."""
        if self._host_error is not None:
            ex, self._host_error = self._host_error, None
            raise ex
        _check(rc)

    # ------------------------------------------------------------- eval
    def encode(self, boards):
        b = np.ascontiguousarray(boards, np.int8).reshape(-1, self.height, self.width)
        state = np.zeros(b.shape + (4,), np.float32)
        mask = np.zeros((len(b), self.action_space), np.uint8)
        _check(self._L.az_encode(self._h, _ptr(b), len(b), _ptr(state), _ptr(mask)))
        return state, mask.astype(bool)

    def forward(self, x):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, self.height, self.width, 4)
        probs = np.zeros((len(x), self.action_space), np.float32)
        values = np.zeros(len(x), np.float32)
        _check(self._L.az_forward(self._h, _ptr(x), len(x), _ptr(probs), _ptr(values)))
        return probs, values

    # ------------------------------------------------------------- self-play
    def selfplay_begin(self, first_game, n_games, base_seed):
        _check(self._L.az_selfplay_begin(self._h, int(first_game), int(n_games),
                                         int(base_seed) & 0xFFFFFFFF))
        self._n_games = int(n_games)

    def selfplay_step(self, n_moves=1, sync=True):
        """Enqueue n_moves moves for every slot.  sync=False returns at once
        (no stats): the moves run while the caller drains earlier ones --
        selfplay_drain then returns the games of the newest move whose
        snapshot is complete and waits at most for the move before the
        running one (az_selfplay_step with st = NULL)."""
        if not sync:
            self._search_call(self._L.az_selfplay_step(self._h, int(n_moves), None))
            return None
        st = Stats()
        self._search_call(self._L.az_selfplay_step(self._h, int(n_moves), ctypes.byref(st)))
        return st.as_dict()

    def selfplay_run(self, first_game, n_games, base_seed):
        st = Stats()
        self._search_call(self._L.az_selfplay_run(self._h, int(first_game), int(n_games),
                                                  int(base_seed) & 0xFFFFFFFF, ctypes.byref(st)))
        self._n_games = int(n_games)
        return st.as_dict()

    def selfplay_results(self):
        G, P, A = self._n_games, self.height * self.width, self.action_space
        lengths = np.zeros(G, np.int32)
        results = np.zeros(G, np.int32)
        expansions = np.zeros(G, np.int32)
        boards = np.zeros((G, P, self.height, self.width), np.int8)
        policies = np.zeros((G, P, A), np.float64)
        moves = np.zeros((G, P), np.int32)
        _check(self._L.az_selfplay_results(self._h, _ptr(lengths), _ptr(results), _ptr(expansions),
                                           _ptr(boards), _ptr(policies), _ptr(moves)))
        return dict(lengths=lengths, results=results, expansions=expansions, boards=boards,
                    policies=policies, moves=moves)

    def selfplay_drain(self, max_games=None, chunk=4096):
        """Games finished since the previous drain, copied to the host (the
        samples of a running batch, az_selfplay_drain): dict of arrays with
        a leading game axis plus `game_ids` (finish order).  Drained in
        chunks of `chunk` games, so a call allocates for what it returns, not
        for the whole batch."""
        left = int(max_games if max_games is not None else max(self._n_games, 1))
        P, A = self.height * self.width, self.action_space
        parts = []
        while left > 0:
            G = min(chunk, left)
            n = ctypes.c_int64(0)
            out = dict(game_ids=np.zeros(G, np.int64), lengths=np.zeros(G, np.int32),
                       results=np.zeros(G, np.int32), expansions=np.zeros(G, np.int32),
                       boards=np.zeros((G, P, self.height, self.width), np.int8),
                       policies=np.zeros((G, P, A), np.float64), moves=np.zeros((G, P), np.int32))
            _check(self._L.az_selfplay_drain(self._h, G, ctypes.byref(n), *(_ptr(out[k]) for k in (
                "game_ids", "lengths", "results", "expansions", "boards", "policies", "moves"))))
            k = int(n.value)
            parts.append({key: v[:k] for key, v in out.items()} if k < G else out)
            left -= k
            if k < G:
                break
        if len(parts) == 1:
            p = parts[0]
            return {key: (v.copy() if v.base is not None else v) for key, v in p.items()}
        return {key: np.concatenate([p[key] for p in parts]) for key in parts[0]}

    # ------------------------------------------------------------- tree API
    def tree_reset(self, slots, boards):
        slots = np.ascontiguousarray(slots, np.int32)
        b = np.ascontiguousarray(boards, np.int8).reshape(len(slots), self.height, self.width)
        _check(self._L.az_tree_reset(self._h, len(slots), _ptr(slots), _ptr(b)))

    def tree_release(self, slots):
        slots = np.ascontiguousarray(slots, np.int32)
        _check(self._L.az_tree_release(self._h, len(slots), _ptr(slots)))

    def tree_search(self, n_sims, noise=None):
        """noise (engines made with dirichlet_noise): [slots, rows, A] float64,
        row r of slot s the np.random.dirichlet vector its r-th root selection
        mixes in (az_tree_search_noise)."""
        if noise is None:
            self._search_call(self._L.az_tree_search(self._h, int(n_sims)))
            return
        noise = np.ascontiguousarray(noise, np.float64)
        if noise.ndim != 3 or noise.shape[0] != self.slots or noise.shape[2] != self.action_space:
            raise ValueError(f"noise must be [slots={self.slots}, rows, A={self.action_space}], got {noise.shape}")
        self._search_call(self._L.az_tree_search_noise(self._h, int(n_sims), _ptr(noise), int(noise.shape[1])))

    def tree_play(self, uniforms=None, greedy=False, deterministic=False):
        S, A = self.slots, self.action_space
        u = None if deterministic else np.ascontiguousarray(uniforms, np.float64).reshape(S)
        moves = np.zeros(S, np.int32)
        status = np.zeros(S, np.int32)
        policy = np.zeros((S, A), np.float64)
        _check(self._L.az_tree_play(self._h, _ptr(u), int(bool(greedy)), int(bool(deterministic)),
                                    _ptr(moves), _ptr(status), _ptr(policy)))
        return moves, status, policy

    def tree_info(self, slot):
        """The slot's tree header alone (az_tree_info: no edge copy)."""
        info = np.zeros(5, np.int64)
        rv = np.zeros(1, np.float32)
        _check(self._L.az_tree_info(self._h, int(slot), _ptr(info), _ptr(rv)))
        return dict(arena_top=int(info[0]), root_first=int(info[1]), root_n=int(info[2]), ply=int(info[3]),
                    active=bool(info[4]), root_value=float(rv[0]))

    def tree_export(self, slot):
        info = np.zeros(5, np.int64)
        rv = np.zeros(1, np.float32)
        _check(self._L.az_tree_info(self._h, int(slot), _ptr(info), _ptr(rv)))
        n = int(info[0])
        out = {
            "prior": np.zeros(n, np.float64), "w": np.zeros(n, np.float64),
            "n": np.zeros(n, np.int32), "child": np.zeros(n, np.int32),
            "child_n": np.zeros(n, np.int32), "action": np.zeros(n, np.int32),
            "child_value": np.zeros(n, np.float32),
        }
        _check(self._L.az_tree_export(self._h, int(slot), _ptr(out["prior"]), _ptr(out["w"]),
                                      _ptr(out["n"]), _ptr(out["child"]), _ptr(out["child_n"]),
                                      _ptr(out["action"]), _ptr(out["child_value"])))
        out.update(arena_top=n, root_first=int(info[1]), root_n=int(info[2]), ply=int(info[3]),
                   active=bool(info[4]), root_value=float(rv[0]))
        return out

    # ------------------------------------------------------------- misc
    def stats(self):
        st = Stats()
        _check(self._L.az_stats_get(self._h, ctypes.byref(st)))
        return st.as_dict()

    def cache_clear(self):
        _check(self._L.az_cache_clear(self._h))

    def cache_enable(self, on=True):
        _check(self._L.az_cache_enable(self._h, int(bool(on))))

    def timer(self, on, tree=False, every=1):
        """HIP-event timing of the network launches (az_stats conv_*); tree:
        the select and expand launches too; every >= 3: every `every`-th
        network launch of each lane only (conv_launches counts those)."""
        if every not in (1,) and every < 3:
            raise ValueError("every: 1 or >= 3")
        _check(self._L.az_timer_enable(self._h, (every if every >= 3 else 2 if tree else 1) if on else 0))

    def pow_table(self, n):
        out = np.zeros(int(n), np.float64)
        _check(self._L.az_pow_table(self._h, _ptr(out), int(n)))
        return out


class ChessEngine:
    """libaz chess self-play engine (include/az_chess.h): `slots` concurrent
    chess games on one device, MCTS with the policy/value network on the
    (8, 8, 118) Board.full_state planes and the 1880-move action space."""

    ACTIONS = 1880
    MAX_MOVES = 256

    def __init__(self, mcts_iterations=800, slots=256, evaluator=EVAL_NETWORK, max_plies=512,
                 index_move_greedy=8, exploration_constant=1.5, filters=128, depth=4,
                 value_hidden=256, bn_epsilon=1e-3, arena_edges=0, conv_algo=CONV_F16X2,
                 device=0, lanes=0, cache_log2=0):
        L = load_library()
        self.slots, self.mcts_iterations = slots, mcts_iterations
        self.max_plies = max_plies if max_plies > 0 else 512
        cfg = ChessConfig(mcts_iterations=mcts_iterations, index_move_greedy=index_move_greedy,
                          exploration_constant=exploration_constant, slots=slots,
                          evaluator=evaluator, filters=filters, depth=depth,
                          value_hidden=value_hidden, max_plies=max_plies, bn_epsilon=bn_epsilon,
                          arena_edges=arena_edges, conv_algo=conv_algo, lanes=lanes, cache_log2=cache_log2)
        handle = ctypes.c_void_p()
        _check(L.az_chess_engine_create(int(device), ctypes.byref(cfg), ctypes.byref(handle)))
        self._h, self._L, self._n_games = handle, L, 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.az_chess_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    def set_weights(self, named):
        arr, n, _keep = tensor_array(named)
        _check(self._L.az_chess_engine_set_weights(self._h, arr, n))

    def forward(self, x):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, 8, 8, 118)
        probs = np.zeros((len(x), self.ACTIONS), np.float32)
        values = np.zeros(len(x), np.float32)
        _check(self._L.az_chess_forward(self._h, _ptr(x), len(x), _ptr(probs), _ptr(values)))
        return probs, values

    def selfplay_begin(self, first_game, n_games, base_seed):
        _check(self._L.az_chess_selfplay_begin(self._h, int(first_game), int(n_games),
                                               int(base_seed) & 0xFFFFFFFF))
        self._n_games = int(n_games)

    def selfplay_step(self, n_moves=1, sync=True):
        """Enqueue n_moves moves for every slot; sync=False returns at once (no
        stats) and selfplay_drain returns the games of the newest move whose
        snapshot is complete (az_chess_selfplay_step with st = NULL, ABI 10)."""
        if not sync:
            _check(self._L.az_chess_selfplay_step(self._h, int(n_moves), None))
            return None
        st = Stats()
        _check(self._L.az_chess_selfplay_step(self._h, int(n_moves), ctypes.byref(st)))
        return st.as_dict()

    def selfplay_drain(self, max_games=None, chunk=64):
        """Games finished since the previous drain (az_chess_selfplay_drain):
        the arrays of selfplay_results with a leading axis over the drained
        games in finish order, plus `game_ids`.  Chunked: a chess game's dense
        rows are ~1.3 MB (max_plies x 256 policy entries)."""
        from custom_alphazero.chess.kernels import POS_DTYPE
        left = int(max_games if max_games is not None else max(self._n_games, 1))
        P, M = self.max_plies, self.MAX_MOVES
        keys = ("game_ids", "lengths", "results", "terminations", "expansions", "positions", "moves",
                "policy_n", "policy_actions", "policy_probs")
        parts = []
        while left > 0:
            G = min(chunk, left)
            n = ctypes.c_int64(0)
            out = dict(game_ids=np.zeros(G, np.int64), lengths=np.zeros(G, np.int32),
                       results=np.zeros(G, np.int32), terminations=np.zeros(G, np.int32),
                       expansions=np.zeros(G, np.int32), positions=np.zeros((G, P), POS_DTYPE),
                       moves=np.zeros((G, P), np.uint16), policy_n=np.zeros((G, P), np.int32),
                       policy_actions=np.zeros((G, P, M), np.int16),
                       policy_probs=np.zeros((G, P, M), np.float64))
            _check(self._L.az_chess_selfplay_drain(self._h, G, ctypes.byref(n), *(_ptr(out[k]) for k in keys)))
            k = int(n.value)
            parts.append({key: v[:k].copy() for key, v in out.items()})
            left -= k
            if k < G:
                break
        return {key: np.concatenate([p[key] for p in parts]) for key in keys}

    def selfplay_run(self, first_game, n_games, base_seed):
        st = Stats()
        _check(self._L.az_chess_selfplay_run(self._h, int(first_game), int(n_games),
                                             int(base_seed) & 0xFFFFFFFF, ctypes.byref(st)))
        self._n_games = int(n_games)
        return st.as_dict()

    def selfplay_results(self, with_samples=True):
        from custom_alphazero.chess.kernels import POS_DTYPE
        G, P, M = self._n_games, self.max_plies, self.MAX_MOVES
        out = {k: np.zeros(G, np.int32) for k in ("lengths", "results", "terminations", "expansions")}
        if with_samples:
            out["positions"] = np.zeros((G, P), POS_DTYPE)
            out["moves"] = np.zeros((G, P), np.uint16)
            out["policy_n"] = np.zeros((G, P), np.int32)
            out["policy_actions"] = np.zeros((G, P, M), np.int16)
            out["policy_probs"] = np.zeros((G, P, M), np.float64)
        g = out.get
        _check(self._L.az_chess_selfplay_results(
            self._h, _ptr(g("lengths")), _ptr(g("results")), _ptr(g("terminations")),
            _ptr(g("expansions")), _ptr(g("positions")), _ptr(g("moves")), _ptr(g("policy_n")),
            _ptr(g("policy_actions")), _ptr(g("policy_probs"))))
        return out

    def stats(self):
        st = Stats()
        _check(self._L.az_chess_stats(self._h, ctypes.byref(st)))
        return st.as_dict()

    def timer(self, on):
        _check(self._L.az_chess_timer_enable(self._h, int(bool(on))))

    # ------------------------------------------------------------- tree API
    def tree_reset(self, slots, roots):
        from custom_alphazero.chess.kernels import POS_DTYPE
        slots = np.ascontiguousarray(slots, np.int32)
        roots = np.ascontiguousarray(roots, POS_DTYPE).reshape(len(slots))
        _check(self._L.az_chess_tree_reset(self._h, len(slots), _ptr(slots), _ptr(roots)))

    def tree_release(self, slots):
        slots = np.ascontiguousarray(slots, np.int32)
        _check(self._L.az_chess_tree_release(self._h, len(slots), _ptr(slots)))

    def tree_search(self, n_sims):
        _check(self._L.az_chess_tree_search(self._h, int(n_sims)))

    def tree_play(self, uniforms=None, greedy=False, deterministic=False):
        """-> moves [S] (move codes, -1 idle), status [S] (AZ_CHESS_* of the new
        root), policy_n [S], policy_actions [S, 256], policy_probs [S, 256]."""
        S, M = self.slots, self.MAX_MOVES
        u = None if deterministic else np.ascontiguousarray(uniforms, np.float64).reshape(S)
        out = dict(moves=np.zeros(S, np.int32), status=np.zeros(S, np.int32),
                   policy_n=np.zeros(S, np.int32), policy_actions=np.zeros((S, M), np.int16),
                   policy_probs=np.zeros((S, M), np.float64))
        _check(self._L.az_chess_tree_play(self._h, _ptr(u), int(bool(greedy)), int(bool(deterministic)),
                                          *(_ptr(out[k]) for k in ("moves", "status", "policy_n",
                                                                   "policy_actions", "policy_probs"))))
        return out

    def tree_export(self, slot):
        info = np.zeros(5, np.int64)
        rv = np.zeros(1, np.float32)
        _check(self._L.az_chess_tree_info(self._h, int(slot), _ptr(info), _ptr(rv)))
        n = int(info[0])
        out = dict(prior=np.zeros(n, np.float64), w=np.zeros(n, np.float64), n=np.zeros(n, np.int32),
                   child=np.zeros(n, np.int32), child_n=np.zeros(n, np.int32),
                   moves=np.zeros(n, np.int32), child_value=np.zeros(n, np.float32))
        _check(self._L.az_chess_tree_export(self._h, int(slot), *(_ptr(out[k]) for k in (
            "prior", "w", "n", "child", "child_n", "moves", "child_value"))))
        out.update(arena_top=n, root_first=int(info[1]), root_n=int(info[2]), ply=int(info[3]),
                   active=bool(info[4]), root_value=float(rv[0]))
        return out
