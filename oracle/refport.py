"""Python port of the reference's self-play loop -- the CPU baseline (TEST INFRASTRUCTURE).

Only bench.py's cpu_baseline leg and tests/ use this module.  It keeps the
reference's *structure* so its speed is the reference's speed (calibration in
BASELINE.md): an object tree with eagerly created child boards (deepcopy per
child, reference mcts.py:151-160), one batch-1 network call per expanded leaf
(mcts.py:130-137), a dict cache keyed by repr(board) (mcts.py:123-142), greedy
play from ply 8 (self_play.py:62).  Arithmetic follows the reference under
its pinned numpy 1.24 (legacy promotion): UCB in float64 with Python's
`** 0.5`, float32 prior normalisation, np.random.choice per move.
tests/test_refport.py pins it against the golden vectors.

The network stand-in is a torch-CPU module with the reference architecture
(TensorFlow 2.7.1 is not installed here); run it with torch.set_num_threads(1)
per worker like the reference's one-game-per-process joblib fan-out.
"""
import time
from copy import deepcopy

import numpy as np

DIRS = ((0, 1), (1, 1), (1, 0), (1, -1))


class PortMove:
    """Move value object with the reference's fields (connect_n/move.py)."""
    __slots__ = ("gravity", "x", "y")

    def __init__(self, gravity, x, y=None):
        self.gravity, self.x, self.y = gravity, x, y

    def __eq__(self, other):
        return (self.x, self.y) == (other.x, other.y)

    def __hash__(self):
        return hash((self.x, self.y))


class PortBoard:
    """Connect-N rules, reference connect_n/board.py:12-268 (canonical mirror).

    Carries the same per-board state as the reference Board (piece tables,
    played Move objects, colour constants) so copying a board costs what the
    reference's deepcopy costs (the dominant CPU cost).
    """

    def __init__(self, height, width, n, gravity):
        self.board_height, self.board_width, self.n, self.gravity = height, width, n, gravity
        self.black, self.empty, self.white = -1, 0, 1
        self.pieces = {-1: "O", 0: ".", 1: "X"}
        self.pieces_to_int = {v: k for k, v in self.pieces.items()}
        self.played_moves = []
        self.array = np.zeros((height, width)).astype("int8")
        self.turn = 1
        self.fullmove_number = 0
        self.game_over = False
        self.is_null = None

    # short aliases used by the search
    @property
    def h(self):
        return self.board_height

    @property
    def w(self):
        return self.board_width

    @property
    def cells(self):
        return self.array

    @cells.setter
    def cells(self, value):
        self.array = value

    @property
    def plies(self):
        return self.fullmove_number

    @property
    def over(self):
        return self.game_over

    def key(self):
        return "\n".join("".join(map(lambda c: self.pieces[c], row)) for row in self.array)

    def moves(self):
        if self.gravity:
            return [PortMove(True, int(x)) for x in np.where(self.array[0, :] == 0)[0]]
        return [PortMove(False, int(x), int(y)) for y, x in zip(*np.where(self.array == 0))]

    def action_of(self, move):
        return move.x if self.gravity else move.x * self.board_height + move.y

    def all_moves(self):
        if self.gravity:
            return [PortMove(True, x) for x in range(self.board_width)]
        return [PortMove(False, x, y) for x in range(self.board_width) for y in range(self.board_height)]

    def legal(self):
        """Board.moves order, as action indices (x, or x*H+y without gravity)."""
        return [self.action_of(m) for m in self.moves()]

    def legal_mask(self):
        current = self.moves()
        return np.asarray([m in current for m in self.all_moves()])

    def state(self):
        one_hot = np.eye(3)[self.array]
        return np.dstack([one_hot, np.ones((self.board_height, self.board_width)) * self.turn]).astype("float32")

    def _place(self, action):
        h, w = self.board_height, self.board_width
        if self.gravity:
            x = action
            col = self.array[:, x]
            y = -1
            for r in range(h):
                if col[r] != 0:
                    break
                y = r
        else:
            x, y = action // h, action % h
        self.array[y, x] = self.turn
        for dx, dy in DIRS:
            run = 1
            for s in (1, -1):
                cx, cy = x + s * dx, y + s * dy
                while 0 <= cx < w and 0 <= cy < h and self.array[cy, cx] == self.array[y, x]:
                    run += 1
                    cx, cy = cx + s * dx, cy + s * dy
            if run >= self.n:
                self.game_over, self.is_null = True, False
                return
        if not self.moves():
            self.game_over, self.is_null = True, True

    def play(self, action, on_copy=False):
        if self.game_over:
            return self
        b = deepcopy(self) if on_copy else self
        b._place(action)
        b.fullmove_number += 1
        b.array = np.where(b.array == -1, 1, np.where(b.array == 1, -1, b.array)).astype("int8")
        b.turn = 1
        b.played_moves.append(PortMove(self.gravity, action % self.board_width if self.gravity else action // self.board_height,
                                       None if self.gravity else action % self.board_height))
        return b

    def result(self):
        if not self.game_over:
            return None
        return 0 if self.is_null else 1


def normalize(p):
    s = p.sum()
    if s == 0:
        return np.array([1 / len(p)] * len(p))
    return np.divide(p, s, out=np.zeros_like(p), where=s != 0)


class Edge:
    __slots__ = ("parent", "child", "action", "prior", "visits", "value_sum", "played")

    def __init__(self, parent, child, action, prior):
        self.parent, self.child, self.action = parent, child, action
        self.prior = float(prior)  # legacy promotion: np.float32 scalar -> float64 math
        self.visits = 0
        self.value_sum = 0.0
        self.played = False

    def ucb(self, c=1.5):
        try:
            q = self.value_sum / self.visits
        except ZeroDivisionError:
            q = 0.0
        total = sum(e.visits for e in self.parent.edges)
        return q + c * self.prior * (total ** 0.5) / (1 + self.visits)


class Node:
    __slots__ = ("board", "edges", "value")

    def __init__(self, board):
        self.board = board
        self.edges = []
        self.value = None


class PortMCTS:
    def __init__(self, board, evaluator, cache):
        self.board = deepcopy(board)
        self.root = Node(deepcopy(board))
        self.evaluator = evaluator
        self.cache = cache
        self.expansions = 0

    def _eval(self, board):
        k = board.key()
        hit = self.cache.get(k)
        if hit is None:
            hit = self.evaluator(board)
            self.cache[k] = hit
        return hit

    def _expand(self, node):
        probs, value = self._eval(node.board)
        node.value = value
        priors = normalize(probs[node.board.legal_mask()])
        for prior, action in zip(priors, node.board.legal()):
            child = Node(node.board.play(action, on_copy=True))
            node.edges.append(Edge(node, child, action, prior))
        self.expansions += 1
        return value

    def search(self, sims):
        for _ in range(sims):
            node, path = self.root, []
            while node.edges:
                scores = [e.ucb() for e in node.edges]
                e = node.edges[int(np.argmax(scores))]
                path.append(e)
                node = e.child
            if not node.board.over:
                v = -self._expand(node)
            else:
                v = node.board.result()
            for e in reversed(path):
                e.visits += 1
                e.value_sum += v
                v = -v

    def play(self, greedy, n_actions):
        node = self.root
        visits = [e.visits for e in node.edges]
        if greedy:
            p = np.zeros(len(node.edges)).astype(float)
            p[int(np.argmax(visits))] = 1.0
        else:
            p = normalize(np.asarray(visits).astype(float))
        e = np.random.choice(node.edges, 1, p=p).item()
        e.played = True
        parent_state = self.board.state()
        self.board.play(e.action)
        self.root = e.child
        policy = np.zeros(n_actions)
        policy[[x.action for x in node.edges]] = p
        return parent_state, policy, e.action


def play_game(height, width, n, gravity, sims, seed, evaluator, greedy_ply=8, cache=None):
    """self_play.play_game (self_play.py:37-82) with an explicit seed."""
    np.random.seed(int(seed) % (2 ** 32 - 1))
    # best_saved_model -> PolicyValueModel.__init__'s dummy forward on
    # np.random.rand(1, *input_dim) (model/tensorflow/model.py:167-169)
    np.random.rand(1, height, width, 4)
    A = width if gravity else width * height
    mcts = PortMCTS(PortBoard(height, width, n, gravity), evaluator, {} if cache is None else cache)
    states, policies, moves = [], [], []
    while not mcts.board.over:
        mcts.search(sims)
        s, p, a = mcts.play(mcts.board.plies >= greedy_ply, A)
        states.append(s)
        policies.append(p)
        moves.append(a)
    reward = mcts.board.result()
    rewards = np.repeat(reward, len(states))
    rewards[-2::-2] = -rewards[-2::-2]
    return dict(states=np.asarray(states), policies=np.asarray(policies), rewards=rewards,
                moves=np.asarray(moves), expansions=mcts.expansions, T=len(states))


# ----------------------------------------------------------------- evaluators
class SynthEval:
    def __init__(self, action_space):
        import synth
        self._synth = synth
        self.A = action_space

    def __call__(self, board):
        own, opp = self._synth.masks_from_array(board.cells, board.w)
        p, v = self._synth.synth_eval(own, opp, self.A)
        return np.asarray(p, np.float32), float(np.float32(v))


class TorchCPUNet:
    """Reference architecture on torch-CPU (stand-in for the Keras model),
    batch-1 calls like mcts.py:131-137; weights in Keras layout."""

    def __init__(self, weights, depth, eps=1e-3):
        import torch
        self.torch = torch
        self.depth = depth

        def conv(unit):
            k = torch.tensor(weights[unit + ".kernel"]).permute(3, 2, 0, 1).contiguous()
            g = torch.tensor(weights[unit + ".gamma"])
            sc = g / torch.sqrt(torch.tensor(weights[unit + ".var"]) + eps)
            b = (torch.tensor(weights[unit + ".bias"]) - torch.tensor(weights[unit + ".mean"])) * sc \
                + torch.tensor(weights[unit + ".beta"])
            return k * sc[:, None, None, None], b

        self.stem = conv("stem")
        self.blocks = [(conv(f"block{d}.conv1"), conv(f"block{d}.conv2"), conv(f"block{d}.res"))
                       for d in range(depth)]
        self.pc, self.vc = conv("policy.conv"), conv("value.conv")
        t = lambda n: torch.tensor(weights[n])  # noqa: E731
        self.pd = (t("policy.dense.kernel"), t("policy.dense.bias"))
        self.v1 = (t("value.dense1.kernel"), t("value.dense1.bias"))
        self.v2 = (t("value.dense2.kernel"), t("value.dense2.bias"))

    def __call__(self, board):
        return self.forward_state(board.state())

    def forward_state(self, state):
        """One [H, W, C] state (batch 1) -> (probs [A], value)."""
        torch = self.torch
        F = torch.nn.functional
        with torch.no_grad():
            x = torch.from_numpy(np.ascontiguousarray(state, np.float32)).permute(2, 0, 1)[None]
            h = F.relu(F.conv2d(x, *self.stem, padding=1))
            for c1, c2, r in self.blocks:
                a = F.relu(F.conv2d(h, *c1, padding=1))
                a = F.conv2d(a, *c2, padding=1)
                h = F.relu(a + F.conv2d(h, *r))
            p = F.relu(F.conv2d(h, *self.pc)).permute(0, 2, 3, 1).reshape(1, -1)
            p = torch.softmax(p @ self.pd[0] + self.pd[1], dim=1)
            v = F.relu(F.conv2d(h, *self.vc)).permute(0, 2, 3, 1).reshape(1, -1)
            v = F.relu(v @ self.v1[0] + self.v1[1])
            v = torch.tanh(v @ self.v2[0] + self.v2[1])
        return p.numpy().ravel(), v.numpy().item()


def baseline_worker(args):
    """One CPU worker: plays games until `budget_s` elapses (a game in progress
    finishes).  `cache` is the plays_inferences the reference hands every
    worker (utils.py:38-39): a multiprocessing Manager dict shared by all
    workers when it fans out, or None for the mono-process path (a plain
    dict kept across this worker's games).  Returns (games, expansions,
    seconds)."""
    (height, width, n, gravity, sims, weights, depth, budget_s, seed, cache) = args
    import torch
    torch.set_num_threads(1)
    net = TorchCPUNet(weights, depth)
    t0 = time.perf_counter()
    games = expansions = 0
    if cache is None:
        cache = {}
    while time.perf_counter() - t0 < budget_s:
        r = play_game(height, width, n, gravity, sims, seed + games, net, cache=cache)
        games += 1
        expansions += r["expansions"]
    return games, expansions, time.perf_counter() - t0


class _Budget(Exception):
    pass


def chess_baseline_worker(args):
    """CPU baseline for chess (BASELINE configs[4]): the oracle's chess MCTS
    (C tree, python-chess order, reference arithmetic) with the torch-CPU
    network called at batch 1 on Board.full_state, one thread per worker.
    The reference itself cannot run chess under MCTS and
    its python-chess object tree would be slower than this C tree, so this is
    a generous stand-in.  A game at 800 sims/move outlasts the budget, so the
    worker reports expansions (network calls) and plies completed.
    Returns (expansions, plies, seconds)."""
    (sims, weights, depth, budget_s, seed) = args
    import torch

    import chess_oracle as C
    torch.set_num_threads(1)
    net = TorchCPUNet(weights, depth)
    t0 = time.perf_counter()
    calls = [0]

    def cb(pos, initial):
        if time.perf_counter() - t0 > budget_s:
            raise _Budget()
        calls[0] += 1
        x = C.full_state(*C.reference_history(pos, bool(initial)), pos)
        return net.forward_state(x)

    try:
        C.play_game(sims, seed, 512, callback=cb)
    except _Budget:
        pass
    el = time.perf_counter() - t0
    return calls[0], calls[0] / max(sims, 1), el
