"""MCTS with the reference's API (custom_alphazero/mcts/mcts.py:22-222), run by libaz.

`MCTS.search(n)` runs n PUCT simulations on the GPU (select -> network or
synthetic evaluation -> expand + backup, csrc/az_tree.hip); `MCTS.play(...)`
commits a move there too.  The only host-side randomness is the one
`np.random.random_sample()` draw that the reference's `np.random.choice`
consumes per move (mcts.py:201), taken from the same global numpy stream, so
a caller seeding np.random gets the reference's move sequence bit for bit.

`root` / `current_root` are read-only UCTNode/UCTEdge views exported from the
device arena (the reference's objects, mcts.py:22-85, for visualisation and
inspection; mutating them does not change the search).

A chess Board (custom_alphazero.chess.board.Board) selects ChessMCTS: the
same API over az_chess_tree_* (csrc/az_chess_mcts.hip).  The chess arena
keeps only the live tree (play() compacts the chosen child's subtree into
the other arena half), so there `root` is the tree under the current root.
"""
from copy import deepcopy
from typing import List, Optional, Tuple, Union

import numpy as np

from custom_alphazero import engine as az
from custom_alphazero.config import (ConfigConnectN, ConfigMCTS, ConfigModel, ConfigSelfPlay,
                                     check_mcts_config)
from custom_alphazero.connect_n.board import Board
from custom_alphazero.connect_n.move import Move


class SyntheticEvaluator:
    """Marker model: evaluate leaves with oracle/synth.py's exact function
    (compiled into libaz) instead of a network -- used for parity runs."""


class UCTEdge:
    """Read-only view of one device edge (reference mcts.py:22-55)."""

    def __init__(self, parent, child, action, prior, visit_count, total_action_value):
        self.parent = parent
        self.child = child
        self.action = action
        self.prior = prior
        self.visit_count = visit_count
        self.total_action_value = total_action_value
        self.played = False
        self.greedily_played = False

    @property
    def siblings(self):
        return [e for e in self.parent.edges if e is not self]

    def exploitation_term(self) -> float:
        return self.total_action_value / self.visit_count if self.visit_count else 0.0

    def exploration_term(self, override_prior: Optional[float] = None) -> float:
        prior = float(self.prior if override_prior is None else override_prior)
        total = sum(e.visit_count for e in self.parent.edges)
        return ConfigMCTS.exploration_constant * prior * (total ** 0.5) / (1 + self.visit_count)

    def upper_confidence_bound(self, override_prior: Optional[float] = None) -> float:
        return self.exploitation_term() + self.exploration_term(override_prior)


class UCTNode:
    """Read-only view of an expanded (or leaf) node (reference mcts.py:58-85)."""

    def __init__(self, board_fn, edges=None, evaluated_value=None):
        self._board_fn = board_fn
        self._board = None
        self.edges: List[UCTEdge] = edges if edges is not None else []
        self.evaluated_value = evaluated_value

    @property
    def board(self) -> Board:
        if self._board is None:
            self._board = self._board_fn()
        return self._board

    def get_best_edge(self) -> UCTEdge:
        return self.edges[int(np.argmax([e.upper_confidence_bound() for e in self.edges]))]


def root_noise_rows(rng, k: int, rows: int, A: int) -> np.ndarray:
    """`rows` root-noise vectors as get_best_edge_with_noise draws them
    (mcts.py:74-78: rng.dirichlet(ones(k) * dirichlet_noise_value) for the
    root's k edges), padded to the action space: [max(rows, 1), A]."""
    out = np.zeros((max(rows, 1), A), np.float64)
    alpha = np.ones(k) * ConfigMCTS.dirichlet_noise_value
    for r in range(rows):
        out[r, :k] = rng.dirichlet(alpha)
    return out


def _engine_for(model, all_possible_moves) -> az.Engine:
    c = ConfigConnectN
    if isinstance(model, SyntheticEvaluator):
        evaluator = az.EVAL_SYNTHETIC
    elif model is not None and hasattr(model, "engine_weights"):
        evaluator = az.EVAL_NETWORK
    elif callable(model):
        # any other model is called as the reference calls it (mcts.py:130-137):
        # model(x) -> (probabilities, value), here with every leaf of a simulation in x
        evaluator = az.EVAL_HOST
    else:
        raise TypeError(
            "MCTS on the MI355X engine needs a model (a custom_alphazero PolicyValueModel, "
            "SyntheticEvaluator or any callable model(x) -> (probabilities, value)); HTTP "
            "inference and the exact solver are not on the device path")
    A = len(all_possible_moves)
    sims = max(ConfigSelfPlay.mcts_iterations, 1)
    HW = c.board_height * c.board_width
    eng = az.Engine(c.board_height, c.board_width, c.n, c.gravity, sims, slots=1,
                    evaluator=evaluator, index_move_greedy=ConfigMCTS.index_move_greedy,
                    exploration_constant=ConfigMCTS.exploration_constant,
                    filters=ConfigModel.filters, depth=ConfigModel.depth,
                    value_hidden=ConfigModel.value_hidden, bn_epsilon=ConfigModel.bn_epsilon,
                    arena_edges=max(sims, 1024) * HW * A, max_tree_visits=max(sims, 1024) * HW + 2,
                    dirichlet_noise=ConfigMCTS.enable_dirichlet_noise,
                    dirichlet_alpha=ConfigMCTS.dirichlet_noise_value,
                    dirichlet_ratio=ConfigMCTS.dirichlet_noise_ratio)
    if evaluator == az.EVAL_NETWORK:
        eng.set_weights(model.engine_weights())
    elif evaluator == az.EVAL_HOST:
        eng.set_host_evaluator(model)
    return eng


class MCTS:
    def __new__(cls, board=None, *args, **kwargs):
        if cls is MCTS and _is_chess_board(board):
            return super().__new__(ChessMCTS)
        return super().__new__(cls)

    def __init__(self, board: Board, all_possible_moves: List[Move], concurrency: bool = False,
                 plays_inferences: Optional[dict] = None, model=None, use_solver: bool = False):
        if use_solver:
            raise NotImplementedError("the exact solver (c4solver) is not on the device path")
        self.board = deepcopy(board)
        self.all_possible_moves = all_possible_moves
        self.concurrency = concurrency
        # The reference's (repr(board) -> outputs) cache is transparent to the
        # search (deterministic evaluator); accepted for API compatibility.
        self.plays_inferences = plays_inferences
        self.model = model
        self.use_solver = use_solver
        self._action_index = {m.key(): i for i, m in enumerate(all_possible_moves)}
        self._engine = _engine_for(model, all_possible_moves)
        self._engine.tree_reset([0], self.board.array[None])
        self._root_board = deepcopy(self.board)
        self._played = []  # (global edge index, greedy)
        self.path_cache = []

    # ------------------------------------------------------------ search
    def search(self, iterations_number: int):
        check_mcts_config()
        if self.board.is_game_over():
            return
        n = int(iterations_number)
        if not ConfigMCTS.enable_dirichlet_noise:
            self._engine.tree_search(n)
            return
        # get_best_edge_with_noise (mcts.py:70-85): every select whose root
        # has edges draws np.random.dirichlet from the global stream -- all n
        # selections, or n - 1 when the first one expands the root (:111-120);
        # nothing else in a search draws, so drawing them up front takes the
        # same words in the same order
        expanded = self._engine.tree_info(0)["root_n"] > 0
        rows = n if expanded else max(n - 1, 0)
        noise = root_noise_rows(np.random, len(self.board.moves), rows, len(self.all_possible_moves))
        self._engine.tree_search(n, noise=noise[None])

    def play(self, greedy: bool = False, return_details: bool = False,
             deterministic: bool = False) -> Union[Tuple[np.ndarray, np.ndarray, np.ndarray, Move], Board]:
        before = self._engine.tree_export(0) if not deterministic else None
        u = None if deterministic else np.array([np.random.random_sample()])
        moves, status, policy = self._engine.tree_play(u, greedy=greedy,
                                                       deterministic=deterministic)
        action = int(moves[0])
        if action < 0:
            raise RuntimeError("play() on a finished game")
        move = self.all_possible_moves[action]
        if before is None:
            before = self._engine.tree_export(0)
        f, k = before["root_first"], before["root_n"]
        for i in range(f, f + k):
            if before["action"][i] == action:
                self._played.append((i, bool(greedy)))
                break
        parent_state = self.board.full_state
        self.board.play(move, keep_same_player=True)
        child_state = self.board.full_state
        if return_details:
            return parent_state, child_state, policy[0].copy(), move
        return self.board

    # ------------------------------------------------------------ tree views
    def _build(self, current=False):
        t = self._engine.tree_export(0)
        played = dict(self._played)
        moves = self.all_possible_moves

        def make_node(first, count, value, board_fn):
            node = UCTNode(board_fn, evaluated_value=value)
            for i in range(first, first + count):
                child_fn = (lambda parent=node, a=int(t["action"][i]):
                            parent.board.play(moves[a], on_copy=True, keep_same_player=True))
                if t["child"][i] >= 0:
                    child = make_node(int(t["child"][i]), int(t["child_n"][i]),
                                      float(t["child_value"][i]), child_fn)
                else:
                    child = UCTNode(child_fn)
                e = UCTEdge(node, child, moves[int(t["action"][i])], float(t["prior"][i]),
                            int(t["n"][i]), float(t["w"][i]))
                if i in played:
                    e.played, e.greedily_played = True, played[i]
                node.edges.append(e)
            return node

        if current:
            board = deepcopy(self.board)
            return make_node(t["root_first"], t["root_n"], t["root_value"], lambda: board)
        root_board = deepcopy(self._root_board)
        n0 = len(root_board.moves) if t["arena_top"] else 0
        return make_node(0, n0, None, lambda: root_board)

    @property
    def root(self) -> UCTNode:
        return self._build(current=False)

    @property
    def current_root(self) -> UCTNode:
        return self._build(current=True)


# ---------------------------------------------------------------- chess
def _is_chess_board(board) -> bool:
    from custom_alphazero.chess.board import Board as ChessBoard
    return isinstance(board, ChessBoard)


def _chess_engine_for(model):
    from custom_alphazero.config import ConfigSelfPlay as SP
    if isinstance(model, SyntheticEvaluator):
        evaluator = az.EVAL_SYNTHETIC
    elif model is not None and hasattr(model, "engine_weights"):
        evaluator = az.EVAL_NETWORK
    else:
        # the chess engine has no host-evaluator seam (az_chess_config.evaluator
        # is AZ_EVAL_NETWORK or AZ_EVAL_SYNTHETIC): a plain callable model is refused
        raise TypeError(
            "chess MCTS on the MI355X engine needs a custom_alphazero PolicyValueModel or a "
            "SyntheticEvaluator (the chess engine has no host-evaluator seam for other callables)")
    sims = max(SP.mcts_iterations, 1)
    max_plies = max(SP.chess_max_plies, 1)
    # a tree holds at most the visits of its root: sims per search plus the
    # reused subtree; 218 edges bound one expansion, ~40 is typical
    eng = az.ChessEngine(mcts_iterations=sims, slots=1, evaluator=evaluator, max_plies=max_plies,
                         index_move_greedy=ConfigMCTS.index_move_greedy,
                         exploration_constant=ConfigMCTS.exploration_constant,
                         filters=ConfigModel.filters, depth=ConfigModel.depth,
                         value_hidden=ConfigModel.value_hidden, bn_epsilon=ConfigModel.bn_epsilon,
                         arena_edges=160 * sims + 4096)
    if evaluator == az.EVAL_NETWORK:
        eng.set_weights(model.engine_weights())
    return eng


class ChessMCTS(MCTS):
    """MCTS (mcts.py:86-222) with a chess board: search, expansion (network
    on Board.full_state, priors zipped with python-chess's move order),
    backup and play run on the device (az_chess_tree_*).  The root is
    evaluated with the history of a deepcopied board, [0 x 7, start-position
    state] (python-chess copy() re-runs the reference subclass's __init__),
    every later board with [0 x 6, start state, board]."""

    def __init__(self, board, all_possible_moves, concurrency: bool = False,
                 plays_inferences: Optional[dict] = None, model=None, use_solver: bool = False):
        from custom_alphazero.chess.utils import get_all_possible_moves
        if use_solver:
            raise NotImplementedError("the exact solver (c4solver) is not on the device path")
        canonical = get_all_possible_moves()
        if [m.uci for m in all_possible_moves] != [m.uci for m in canonical]:
            raise ValueError("chess MCTS on the device uses get_all_possible_moves() (1880 moves, "
                             "Move order) as the action space")
        self.board = deepcopy(board)
        self.all_possible_moves = all_possible_moves
        self.concurrency = concurrency
        self.plays_inferences = plays_inferences
        self.model = model
        self.use_solver = use_solver
        self._engine = _chess_engine_for(model)
        self._engine.tree_reset([0], self.board._pos[None])
        self.path_cache = []

    def search(self, iterations_number: int):
        check_mcts_config("chess")
        if self.board.is_game_over():
            return
        self._engine.tree_search(int(iterations_number))

    def play(self, greedy: bool = False, return_details: bool = False, deterministic: bool = False):
        if self.board.is_game_over():
            raise RuntimeError("play() on a finished game")
        u = None if deterministic else np.array([np.random.random_sample()])
        out = self._engine.tree_play(u, greedy=greedy, deterministic=deterministic)
        code = int(out["moves"][0])
        if code < 0:
            raise RuntimeError("play() on a finished game")
        from custom_alphazero.chess.move import Move as ChessMove
        move = ChessMove.from_code(code)
        parent_state = self.board.full_state
        self.board.play(move, keep_same_player=True)
        child_state = self.board.full_state
        if return_details:
            policy = np.zeros(len(self.all_possible_moves))
            k = int(out["policy_n"][0])
            policy[out["policy_actions"][0, :k].astype(np.int64)] = out["policy_probs"][0, :k]
            return parent_state, child_state, policy, move
        return self.board

    def _build(self, current=False):
        from custom_alphazero.chess.move import Move as ChessMove
        t = self._engine.tree_export(0)

        def make_node(first, count, value, board_fn):
            node = UCTNode(board_fn, evaluated_value=value)
            for i in range(first, first + count):
                mv = ChessMove.from_code(int(t["moves"][i]))
                child_fn = (lambda parent=node, m=mv:
                            parent.board.play(m, on_copy=True, keep_same_player=True))
                if t["child"][i] >= 0:
                    child = make_node(int(t["child"][i]), int(t["child_n"][i]),
                                      float(t["child_value"][i]), child_fn)
                else:
                    child = UCTNode(child_fn)
                node.edges.append(UCTEdge(node, child, mv, float(t["prior"][i]), int(t["n"][i]),
                                          float(t["w"][i])))
            return node

        board = deepcopy(self.board)
        value = t["root_value"] if t["root_n"] else None
        return make_node(t["root_first"], t["root_n"], value, lambda: board)

    @property
    def root(self) -> UCTNode:
        return self._build()

    @property
    def current_root(self) -> UCTNode:
        return self._build(current=True)
