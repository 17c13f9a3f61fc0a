"""Arena: two models play each other (reference evaluation/evaluate.py:29-134).

* `_single_game_evaluation` / `evaluate_two_models` keep the reference's
  signatures and game loop (one game at a time; per-move fresh MCTS with the
  model to move, or the raw policy when evaluate_with_mcts is False).
* `evaluate_two_models_batched` plays all evaluation games at once on the
  device: one engine per model, each ply every unfinished game is searched by
  the engine of the model to move (az_tree_reset / az_tree_release keep the
  other engine's copy idle).  With deterministic=True the per-game results are
  those of the sequential loop; with stochastic play each game draws from its
  own RandomState(seed + game) instead of the shared np.random stream (the
  only difference; the draw count per move is the reference's).  Dirichlet
  root noise (ConfigMCTS.enable_dirichlet_noise) is drawn the same way: the
  search's root-noise vectors, then play's draw, from the game's stream.
The exact-solver scoring path needs the refused c4solver binary (SURVEY.md
section 8c) and raises NotImplementedError.
"""
from typing import List, Optional, Tuple

import numpy as np

from custom_alphazero import engine as az
from custom_alphazero.config import (ConfigConnectN, ConfigMCTS, ConfigModel, ConfigSelfPlay,
                                     ConfigServing, check_mcts_config)
from custom_alphazero.connect_n.board import Board
from custom_alphazero.connect_n.move import Move
from custom_alphazero.mcts.mcts import MCTS, root_noise_rows
from custom_alphazero.mcts.utils import normalize_probabilities

get_all_possible_moves = Board.get_all_possible_moves


def _policy_move(model, board: Board, all_possible_moves: List[Move], deterministic: bool, rng):
    """evaluate.py:40-53: raw-policy move (legal probabilities normalised)."""
    probabilities, _ = model(np.expand_dims(board.full_state, axis=0))
    probabilities = probabilities.numpy().ravel()
    legal = normalize_probabilities(probabilities[board.legal_moves_mask(all_possible_moves)])
    if deterministic:
        return board.moves[int(np.argmax(legal))]
    return rng.choice(board.moves, 1, p=legal).item()


def _single_game_evaluation(current_model, previous_model, game_index: int,
                            all_possible_moves: List[Move], evaluate_with_mcts: bool,
                            evaluate_with_solver: bool, deterministic: bool,
                            rng=None, trace: Optional[list] = None) -> Tuple[int, Optional[List[float]]]:
    """evaluate.py:29-98.  Additions: `rng` replaces the global np.random;
    `trace` collects the final board's array."""
    if evaluate_with_solver:
        raise NotImplementedError("solver scoring needs the c4solver binary (not run here)")
    rng = np.random if rng is None else rng
    model = current_model if game_index % 2 == 0 else previous_model
    if not evaluate_with_mcts:
        board = Board()
        while not board.is_game_over():
            move = _policy_move(model, board, all_possible_moves, deterministic, rng)
            board.play(move, keep_same_player=True)
            if not board.is_game_over():
                model = previous_model if model is current_model else current_model
    else:
        mcts = MCTS(board=Board(), all_possible_moves=all_possible_moves, concurrency=False,
                    model=model, plays_inferences={})
        while not mcts.board.is_game_over():
            greedy = mcts.board.fullmove_number > ConfigMCTS.index_move_greedy
            if rng is not np.random and (not deterministic or ConfigMCTS.enable_dirichlet_noise):
                # the shim draws (root noise in search, the move in play) from
                # np.random; route this game's stream through it
                state = np.random.get_state()
                np.random.set_state(rng.get_state())
                try:
                    mcts.search(ConfigSelfPlay.mcts_iterations)
                    mcts.play(greedy, deterministic=deterministic)
                finally:
                    rng.set_state(np.random.get_state())
                    np.random.set_state(state)
            else:
                mcts.search(ConfigSelfPlay.mcts_iterations)
                mcts.play(greedy, deterministic=deterministic)
            if not mcts.board.is_game_over():
                model = previous_model if mcts.model is current_model else current_model
                mcts = MCTS(board=mcts.board, all_possible_moves=all_possible_moves,
                            concurrency=False, model=model, plays_inferences={})
        board = mcts.board
    if trace is not None:
        trace.append(board.array.copy())
    result = board.get_result(keep_same_player=True)
    if result:
        return (1 if current_model is model else -1), []
    return 0, []


def _score(results) -> float:
    """evaluate.py:120-134: wins / decisive games, 0.5 when all draws."""
    results = np.asarray(results)
    if np.all(results == 0):
        return 0.5
    return float((results == 1).sum() / (results != 0).sum())


def evaluate_two_models(model, other_model, evaluate_with_mcts: bool = False,
                        evaluate_with_solver: bool = False, deterministic: bool = False):
    """evaluate.py:101-134: (score of `model`, solver score or None)."""
    if evaluate_with_solver:
        raise NotImplementedError("solver scoring needs the c4solver binary (not run here)")
    all_possible_moves = get_all_possible_moves()
    results = [_single_game_evaluation(model, other_model, g, all_possible_moves,
                                       evaluate_with_mcts, False, deterministic)[0]
               for g in range(ConfigServing.evaluation_games_number)]
    return _score(results), None


def _arena_engine(model, n_slots: int) -> az.Engine:
    check_mcts_config()
    c = ConfigConnectN
    eng = az.Engine(c.board_height, c.board_width, c.n, c.gravity,
                    max(ConfigSelfPlay.mcts_iterations, 1), slots=n_slots,
                    evaluator=az.EVAL_NETWORK, index_move_greedy=ConfigMCTS.index_move_greedy,
                    exploration_constant=ConfigMCTS.exploration_constant,
                    filters=ConfigModel.filters, depth=ConfigModel.depth,
                    value_hidden=ConfigModel.value_hidden, bn_epsilon=ConfigModel.bn_epsilon,
                    lanes=1, dirichlet_noise=ConfigMCTS.enable_dirichlet_noise,
                    dirichlet_alpha=ConfigMCTS.dirichlet_noise_value,
                    dirichlet_ratio=ConfigMCTS.dirichlet_noise_ratio)
    eng.set_weights(model.engine_weights())
    return eng


def evaluate_two_models_batched(model, other_model, n_games: Optional[int] = None,
                                evaluate_with_mcts: bool = False, deterministic: bool = True,
                                seed: int = 0, trace: Optional[list] = None):
    """All games at once.  Returns (score of `model`, per-game results);
    `trace` collects the final boards' arrays in game order."""
    n = int(n_games or ConfigServing.evaluation_games_number)
    all_moves = get_all_possible_moves()
    A = len(all_moves)
    boards = [Board() for _ in range(n)]
    side = np.array([g % 2 for g in range(n)])  # 0: `model` to move, 1: `other_model`
    rngs = [np.random.RandomState((seed + g) % 2 ** 32) for g in range(n)]
    models = (model, other_model)
    engines = [_arena_engine(m, n) for m in models] if evaluate_with_mcts else None
    active = [set(), set()]
    last_side = np.zeros(n, np.int64)
    while True:
        live = [g for g in range(n) if not boards[g].is_game_over()]
        if not live:
            break
        ply = boards[live[0]].fullmove_number  # lockstep: every live game is at the same ply
        for s in (0, 1):
            idx = [g for g in live if side[g] == s]
            if not idx:
                continue
            if not evaluate_with_mcts:
                x = np.stack([boards[g].full_state for g in idx])
                probs = models[s](x)[0].numpy()
                for k, g in enumerate(idx):
                    legal = normalize_probabilities(probs[k][boards[g].legal_moves_mask(all_moves)])
                    if deterministic:
                        move = boards[g].moves[int(np.argmax(legal))]
                    else:
                        move = rngs[g].choice(boards[g].moves, 1, p=legal).item()
                    boards[g].play(move, keep_same_player=True)
            else:
                eng = engines[s]
                stale = sorted(active[s] - set(idx))
                if stale:
                    eng.tree_release(stale)
                eng.tree_reset(idx, np.stack([boards[g].array for g in idx]))
                active[s] = set(idx)
                sims = ConfigSelfPlay.mcts_iterations
                if ConfigMCTS.enable_dirichlet_noise:
                    # each move's MCTS starts on an unexpanded root (evaluate.py:64-83):
                    # sims - 1 root selections draw from the game's stream, before play's draw
                    rows = max(sims - 1, 0)
                    noise = np.zeros((n, max(rows, 1), A))
                    for g in idx:
                        noise[g] = root_noise_rows(rngs[g], len(boards[g].moves), rows, A)
                    eng.tree_search(sims, noise=noise)
                else:
                    eng.tree_search(sims)
                u = None
                if not deterministic:
                    u = np.zeros(n)
                    for g in idx:
                        u[g] = rngs[g].random_sample()  # np.random.choice's one draw (mcts.py:201)
                greedy = ply > ConfigMCTS.index_move_greedy
                moves, _status, _policy = eng.tree_play(u, greedy=greedy, deterministic=deterministic)
                for g in idx:
                    boards[g].play(all_moves[int(moves[g])], keep_same_player=True)
            last_side[idx] = s
        side = 1 - side
    results = []
    for g in range(n):
        if trace is not None:
            trace.append(boards[g].array.copy())
        r = boards[g].get_result(keep_same_player=True)
        results.append(0 if not r else (1 if last_side[g] == 0 else -1))
    _ = A
    return _score(results), results
