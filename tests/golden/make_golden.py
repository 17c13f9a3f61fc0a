"""Generate the golden parity fixtures by running the REAL reference here.

Run ONLY in the development container (the reference never travels):

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tests/golden/make_golden.py

Interpreter choice: /opt/conda/bin/python3.9 has numpy 1.26.4, whose legacy
(value-based) promotion matches the reference's pinned numpy 1.24.3
(reference poetry.lock:1163-1164) -- the UCB arithmetic then runs in float64
exactly as the reference shipped.  The default python3 has numpy 2.x (NEP 50)
and would silently change the arithmetic (finding 3).

Two stub modules are inserted before importing the reference:
  * custom_alphazero.model.tensorflow.model -- TensorFlow is not installed.
    Its PolicyValueModel returns oracle/synth.py's exactly-representable
    evaluator, so the fixtures pin the reference's tree arithmetic bit for bit.
  * graphviz -- only used by visualisation code off the hot path.

Everything written is data (.npz arrays, allow_pickle=False loadable).
"""
import math
import os
import random
import sys
import time
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REFERENCE = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "oracle"))
import synth  # noqa: E402

assert np.__version__.startswith("1."), "golden vectors need legacy numpy promotion"


class _Tensor:
    def __init__(self, array):
        self._array = array

    def numpy(self):
        return self._array


class StubPolicyValueModel:
    """Stand-in for model/tensorflow/model.py:152-188: the call signature, and
    the constructor's one use of numpy's global stream -- its dummy forward on
    np.random.rand(1, *input_dim) (model.py:167-169), which play_game runs
    between np.random.seed and the game (self_play.py:45-47)."""

    def __init__(self, input_dim, action_space):
        self.input_dim = input_dim
        self.action_space = action_space
        np.random.rand(1, *self.input_dim).astype("float32")

    def __call__(self, x):
        x = np.asarray(x)
        probs, values = [], []
        for state in x:
            own, opp = synth.masks_from_full_state(state)
            p, v = synth.synth_eval(own, opp, self.action_space)
            probs.append(p)
            values.append([v])
        return (
            _Tensor(np.asarray(probs, dtype=np.float32)),
            _Tensor(np.asarray(values, dtype=np.float32)),
        )


def install_stubs():
    model_mod = types.ModuleType("custom_alphazero.model.tensorflow.model")
    model_mod.PolicyValueModel = StubPolicyValueModel
    sys.modules["custom_alphazero.model.tensorflow.model"] = model_mod
    gv = types.ModuleType("graphviz")

    class Digraph:  # noqa: D401 - stub
        def __init__(self, *a, **k):
            pass

    gv.Digraph = Digraph
    sys.modules["graphviz"] = gv
    sys.path.insert(0, REFERENCE)


install_stubs()
os.chdir("/tmp")
from custom_alphazero import config as ref_config  # noqa: E402
from custom_alphazero import self_play as ref_self_play  # noqa: E402
from custom_alphazero.connect_n.board import Board  # noqa: E402
from custom_alphazero.mcts import mcts as ref_mcts  # noqa: E402
from custom_alphazero.mcts.utils import normalize_probabilities  # noqa: E402

ref_config.ConfigGeneral.mono_process = True


def set_game(height, width, n, gravity):
    ref_config.ConfigConnectN.board_height = height
    ref_config.ConfigConnectN.board_width = width
    ref_config.ConfigConnectN.n = n
    ref_config.ConfigConnectN.gravity = gravity


def action_index(move, all_moves):
    return all_moves.index(move)


# ---------------------------------------------------------------- MCTS games
EXPANSIONS = [0]
_orig_expand = ref_mcts.MCTS.evaluate_and_expand


def _counting_expand(self, node):
    EXPANSIONS[0] += 1
    return _orig_expand(self, node)


ref_mcts.MCTS.evaluate_and_expand = _counting_expand


def run_games(name, height, width, n, gravity, sims, seeds, noise=False):
    """noise: ConfigMCTS.enable_dirichlet_noise = True for these games (the
    reference's root Dirichlet noise, mcts.py:70-85, drawn from the game's
    np.random stream at every root selection)."""
    set_game(height, width, n, gravity)
    ref_config.ConfigMCTS.enable_dirichlet_noise = bool(noise)
    all_moves = Board.get_all_possible_moves()
    A = len(all_moves)
    rec = {k: [] for k in (
        "game_len", "expansions", "moves", "greedy", "n_edges", "edge_action",
        "edge_prior", "edge_n", "edge_w", "policy", "state", "reward", "seed")}
    for seed in seeds:
        ref_self_play.time.time = lambda s=seed: float(s)
        EXPANSIONS[0] = 0
        states, policies, rewards, tree = ref_self_play.play_game(
            process_id=0,
            all_possible_moves=all_moves,
            mcts_iterations=sims,
            run_id="golden-fixture",
            plays_inferences={},
        )
        T = len(states)
        node = tree.root
        for ply in range(T):
            edges = node.edges
            played = [e for e in edges if e.played]
            assert len(played) == 1
            ea = np.full(A, -1, np.int32)
            ep = np.zeros(A, np.float64)
            en = np.zeros(A, np.int64)
            ew = np.zeros(A, np.float64)
            for i, e in enumerate(edges):
                ea[i] = action_index(e.action, all_moves)
                ep[i] = float(e.prior)
                en[i] = e.visit_count
                ew[i] = float(e.total_action_value)
            rec["n_edges"].append(len(edges))
            rec["edge_action"].append(ea)
            rec["edge_prior"].append(ep)
            rec["edge_n"].append(en)
            rec["edge_w"].append(ew)
            rec["moves"].append(action_index(played[0].action, all_moves))
            rec["greedy"].append(bool(played[0].greedily_played))
            node = played[0].child
        rec["game_len"].append(T)
        rec["expansions"].append(EXPANSIONS[0])
        rec["policy"].append(np.asarray(policies, np.float64))
        rec["state"].append(np.asarray(states, np.float32))
        rec["reward"].append(np.asarray(rewards, np.int64))
        rec["seed"].append(seed)
    out = dict(
        height=height, width=width, n=n, gravity=gravity, sims=sims, action_space=A,
        seed=np.asarray(rec["seed"], np.uint32),
        game_len=np.asarray(rec["game_len"], np.int64),
        expansions=np.asarray(rec["expansions"], np.int64),
        moves=np.asarray(rec["moves"], np.int64),
        greedy=np.asarray(rec["greedy"], np.bool_),
        n_edges=np.asarray(rec["n_edges"], np.int64),
        edge_action=np.asarray(rec["edge_action"], np.int32),
        edge_prior=np.asarray(rec["edge_prior"], np.float64),
        edge_n=np.asarray(rec["edge_n"], np.int64),
        edge_w=np.asarray(rec["edge_w"], np.float64),
        policy=np.concatenate(rec["policy"]),
        state=np.concatenate(rec["state"]),
        reward=np.concatenate(rec["reward"]),
    )
    out.update(dirichlet_noise=bool(noise), dirichlet_alpha=ref_config.ConfigMCTS.dirichlet_noise_value,
               dirichlet_ratio=ref_config.ConfigMCTS.dirichlet_noise_ratio)
    ref_config.ConfigMCTS.enable_dirichlet_noise = False
    np.savez_compressed(os.path.join(OUT, f"mcts_{name}.npz"), **out)
    print(f"mcts_{name}: {len(seeds)} games, plies={out['game_len'].tolist()}, "
          f"expansions={out['expansions'].tolist()}")


# --------------------------------------------------------------- board rules
def board_playouts(name, height, width, n, gravity, n_games, seed):
    set_game(height, width, n, gravity)
    all_moves = Board.get_all_possible_moves()
    rng = random.Random(seed)
    cols = {k: [] for k in ("game", "move", "array", "game_over", "is_null", "result",
                            "mask", "moves_order", "n_moves", "fullmove")}
    for g in range(n_games):
        board = Board()
        while not board.is_game_over():
            move = rng.choice(board.moves)
            board.play(move, keep_same_player=True)
            mo = np.full(len(all_moves), -1, np.int32)
            order = [action_index(m, all_moves) for m in board.moves]
            mo[: len(order)] = order
            res = board.get_result(keep_same_player=True)
            cols["game"].append(g)
            cols["move"].append(action_index(move, all_moves))
            cols["array"].append(board.array.copy())
            cols["game_over"].append(board.is_game_over())
            cols["is_null"].append(-1 if board.is_null is None else int(board.is_null))
            cols["result"].append(-9 if res is None else res)
            cols["mask"].append(board.legal_moves_mask(all_moves))
            cols["moves_order"].append(mo)
            cols["n_moves"].append(len(order))
            cols["fullmove"].append(board.fullmove_number)
    out = {k: np.asarray(v) for k, v in cols.items()}
    out.update(height=height, width=width, n=n, gravity=gravity)
    np.savez_compressed(os.path.join(OUT, f"board_{name}.npz"), **out)
    print(f"board_{name}: {n_games} playouts, {len(cols['game'])} positions")


# ------------------------------------------------------------------ numerics
def numerics():
    rng = np.random.RandomState(1234)
    ins, outs, lens, out_is64 = [], [], [], []
    for n in range(1, 20):
        for trial in range(40):
            if trial == 0:
                v = np.zeros(n, np.float32)
            else:
                v = (rng.rand(n) * np.exp2(rng.randint(-20, 4, n))).astype(np.float32)
            r = normalize_probabilities(v)
            ins.append(np.pad(v, (0, 19 - n)))
            outs.append(np.pad(np.asarray(r, np.float64), (0, 19 - n)))
            lens.append(n)
            out_is64.append(r.dtype == np.float64)
    # visit-count normalisation (MCTS.play, mcts.py:194-197): float64 input
    vin, vout, vlen = [], [], []
    for n in range(1, 20):
        for trial in range(20):
            c = rng.randint(0, 3000, n).astype(float)
            if trial == 0:
                c[:] = 0
            r = normalize_probabilities(c)
            vin.append(np.pad(c, (0, 19 - n)))
            vout.append(np.pad(r, (0, 19 - n)))
            vlen.append(n)
    # Python `int ** 0.5` (mcts.py:50) vs IEEE sqrt: exceptions below 2e6
    exc = [k for k in range(2_000_001) if k ** 0.5 != math.sqrt(k)]
    exc_val = [k ** 0.5 for k in exc]
    # legacy RandomState: seed -> random_sample, and choice() on policies
    seeds = np.arange(64, dtype=np.uint32)
    uniforms, choices, choice_p = [], [], []
    prng = np.random.RandomState(99)
    for s in seeds:
        np.random.seed(int(s))
        uniforms.append([np.random.random_sample() for _ in range(6)])
        p = prng.randint(0, 50, 7).astype(float)
        p[prng.randint(0, 7)] += 1
        p = normalize_probabilities(p)
        np.random.seed(int(s) + 1000)
        choices.append([int(np.random.choice(np.arange(7), 1, p=p).item()) for _ in range(8)])
        choice_p.append(p)
    np.savez_compressed(
        os.path.join(OUT, "numerics.npz"),
        norm_in=np.asarray(ins, np.float32), norm_out=np.asarray(outs, np.float64),
        norm_len=np.asarray(lens, np.int64), norm_out_is64=np.asarray(out_is64, np.bool_),
        visit_in=np.asarray(vin, np.float64), visit_out=np.asarray(vout, np.float64),
        visit_len=np.asarray(vlen, np.int64),
        pow_exceptions=np.asarray(exc, np.int64), pow_values=np.asarray(exc_val, np.float64),
        mt_seeds=seeds, mt_uniforms=np.asarray(uniforms, np.float64),
        choice_p=np.asarray(choice_p, np.float64), choice_idx=np.asarray(choices, np.int64),
    )
    print(f"numerics: {len(exc)} pow exceptions (first {exc[:5]})")


if __name__ == "__main__":
    t0 = time.time()
    which = sys.argv[1:] or ["numerics", "boards", "mcts"]
    if "numerics" in which:
        numerics()
    if "boards" in which:
        board_playouts("c4", 6, 7, 4, True, 200, 7)
        board_playouts("c5_9x9", 9, 9, 5, True, 60, 8)
        board_playouts("nograv_5x5", 5, 5, 4, False, 80, 9)
    if "mcts" in which:
        run_games("c4_s25", 6, 7, 4, True, 25, list(range(16)))
        run_games("c4_s100", 6, 7, 4, True, 100, list(range(100, 108)))
        run_games("c4_s200", 6, 7, 4, True, 200, list(range(200, 203)))
        run_games("c4_s400", 6, 7, 4, True, 400, [400, 401])
        run_games("c5_9x9_s50", 9, 9, 5, True, 50, [900, 901, 902])
        run_games("nograv_5x5_s25", 5, 5, 4, False, 25, [500, 501, 502, 503])
        run_games("c4_s1", 6, 7, 4, True, 1, [10, 11])
        run_games("c4_s2", 6, 7, 4, True, 2, [20, 21])
    if "mcts" in which or "noise" in which:
        # Dirichlet root noise on (config.py:52-54 with enable_dirichlet_noise = True)
        run_games("c4_s25_noise", 6, 7, 4, True, 25, list(range(30, 38)), noise=True)
        run_games("c4_s100_noise", 6, 7, 4, True, 100, [130, 131, 132], noise=True)
        run_games("c5_9x9_s50_noise", 9, 9, 5, True, 50, [930, 931], noise=True)
        run_games("nograv_5x5_s25_noise", 5, 5, 4, False, 25, [530, 531, 532], noise=True)
    print(f"done in {time.time() - t0:.1f}s")
