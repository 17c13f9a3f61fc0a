"""Self-play worker entrypoints with the reference's signatures
(custom_alphazero/self_play.py:37-119).

* play_game(...) plays ONE game through the MCTS API exactly like the
  reference loop (seeded np.random, search, greedy from ply 8, alternating
  rewards), so it is a drop-in for callers that want the tree back.
* play(...) is the batched path: ConfigSelfPlay.games_per_call games run on
  the device at once (ConfigSelfPlay.concurrent_games trees in flight, slots
  refilled as games end), replacing the reference's one-game-per-process
  joblib fan-out (self_play.py:98-110).  Game g is the reference's play_game
  under np.random.seed(base_seed + g): MT19937(base_seed + g) past the
  2 H W 4 words its model construction draws (az_config.rng_skip).
"""
import json
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from custom_alphazero import engine as az
from custom_alphazero.config import (ConfigConnectN, ConfigGeneral, ConfigMCTS, ConfigModel,
                                     ConfigPath, ConfigSelfPlay, check_mcts_config)
from custom_alphazero.connect_n.board import Board
from custom_alphazero.connect_n.move import Move
from custom_alphazero.mcts.mcts import MCTS, SyntheticEvaluator
from custom_alphazero.utils import best_saved_model, input_dim

get_all_possible_moves = Board.get_all_possible_moves


def alternating_rewards(result: int, length: int) -> np.ndarray:
    """self_play.py:71-78: the final result for the last mover, negated every
    other ply going back, times discounting_factor ** distance."""
    rewards = np.repeat(result, length)
    rewards[-2::-2] = -rewards[-2::-2]
    return rewards * ConfigSelfPlay.discounting_factor ** np.arange(length)[::-1]


def play_game(process_id: int, all_possible_moves: List[Move], mcts_iterations: int, run_id: str,
              plays_inferences: Optional[Dict[str, Tuple[np.ndarray, float]]] = None,
              model=None) -> Tuple[np.ndarray, np.ndarray, np.ndarray, MCTS]:
    seed = int((process_id + 1) * time.time()) % (2 ** 32 - 1)
    np.random.seed(seed)
    if model is None:
        model = best_saved_model(run_id)  # its constructor draws np.random.rand(1, *input_dim)
    else:
        # a caller's model: take the draws the reference's model construction
        # makes at this point (model/tensorflow/model.py:167-169), whatever the
        # game, so the stream after them -- chess's game seed below included --
        # does not depend on whether a model was passed
        np.random.rand(1, *input_dim())
    if ConfigMCTS.enable_dirichlet_noise and ConfigGeneral.game != "chess":
        # root noise draws from the game's own stream: the game runs on the
        # batched engine as game 0 of a one-game batch seeded like this
        # process -- MT19937(seed) past the model construction's 2 H W 4 words
        # (az_config.rng_skip), the stream np.random holds here
        states, policies, rewards, records = play(run_id, plays_inferences, model=model, n_games=1,
                                                  base_seed=seed, sims=mcts_iterations)
        return states, policies, rewards, records[0]
    if ConfigGeneral.game == "chess":
        # one game on the chess engine, seeded like the reference's process seed
        seed = int(np.random.randint(0, 2 ** 31 - 1))
        states, policies, rewards, records = play_chess(model, 1, seed, 0, mcts_iterations)
        return states, policies, rewards, records[0]
    mcts = MCTS(board=Board(), all_possible_moves=all_possible_moves,
                concurrency=ConfigGeneral.concurrency, plays_inferences=plays_inferences,
                model=model, use_solver=ConfigMCTS.use_solver)
    states, policies = [], []
    while not mcts.board.is_game_over():
        mcts.search(mcts_iterations)
        greedy = mcts.board.fullmove_number >= ConfigMCTS.index_move_greedy
        parent_state, _child_state, policy, _move = mcts.play(greedy, return_details=True)
        states.append(parent_state)
        policies.append(policy)
    states, policies = np.asarray(states), np.asarray(policies)
    rewards = alternating_rewards(mcts.board.get_result(keep_same_player=True), len(states))
    return states, policies, rewards, mcts


@dataclass
class GameRecord:
    """Per-game summary returned by play() in place of the reference's pickled
    MCTS trees (the device arena is recycled when a slot takes a new game)."""
    game_id: int
    seed: int
    length: int
    result: int
    expansions: int
    moves: np.ndarray


_ENGINES = {}
# The device transposition cache stands for the caller's plays_inferences
# dict (mcts.py:122-143): it lives as long as the same dict object is passed
# (self_play.__main__ keeps one across play() calls) and is emptied when a
# different dict arrives (utils.reset_plays_inferences_dict, self_play.py:
# 145-146) or the weights change (az_engine_set_weights clears it).
_CACHE_OWNER = {"dict": None}


def _batched_engine(model, n_slots, sims=None):
    check_mcts_config("selfplay")
    c = ConfigConnectN
    synthetic = isinstance(model, SyntheticEvaluator)
    sims = int(sims or ConfigSelfPlay.mcts_iterations)
    noise = (bool(ConfigMCTS.enable_dirichlet_noise), ConfigMCTS.dirichlet_noise_value,
             ConfigMCTS.dirichlet_noise_ratio)
    key = (c.board_height, c.board_width, c.n, c.gravity, sims, n_slots,
           synthetic, ConfigMCTS.index_move_greedy, ConfigMCTS.exploration_constant,
           ConfigModel.depth, ConfigSelfPlay.cache_log2, ConfigSelfPlay.lanes, noise)
    eng = _ENGINES.get(key)
    if eng is None:
        eng = az.Engine(c.board_height, c.board_width, c.n, c.gravity, sims, slots=n_slots,
                        evaluator=az.EVAL_SYNTHETIC if synthetic else az.EVAL_NETWORK,
                        index_move_greedy=ConfigMCTS.index_move_greedy,
                        exploration_constant=ConfigMCTS.exploration_constant,
                        filters=ConfigModel.filters, depth=ConfigModel.depth,
                        value_hidden=ConfigModel.value_hidden, bn_epsilon=ConfigModel.bn_epsilon,
                        cache_log2=ConfigSelfPlay.cache_log2, lanes=ConfigSelfPlay.lanes, compact=True,
                        dirichlet_noise=noise[0], dirichlet_alpha=noise[1], dirichlet_ratio=noise[2])
        eng.weights_key = None
        _ENGINES.clear()
        _ENGINES[key] = eng
        _CACHE_OWNER["dict"] = None
    if not synthetic:
        # content hash: play() reloads the best model from disk every call like
        # the reference (utils.py:42-48); unchanged weights keep the cache
        wkey = model.content_hash if hasattr(model, "content_hash") else (id(model), getattr(model, "_version", None))
        if eng.weights_key != wkey:  # new best model: upload (clears the cache)
            eng.set_weights(model.engine_weights())
            eng.weights_key = wkey
    return eng


_CHESS_ENGINES = {}


def _chess_engine(model, n_slots, sims):
    check_mcts_config("chess")
    synthetic = isinstance(model, SyntheticEvaluator)
    key = (sims, n_slots, synthetic, ConfigMCTS.index_move_greedy, ConfigMCTS.exploration_constant,
           ConfigModel.depth, ConfigSelfPlay.chess_max_plies, ConfigSelfPlay.chess_cache_log2)
    eng = _CHESS_ENGINES.get(key)
    if eng is None:
        eng = az.ChessEngine(sims, slots=n_slots,
                             evaluator=az.EVAL_SYNTHETIC if synthetic else az.EVAL_NETWORK,
                             max_plies=ConfigSelfPlay.chess_max_plies,
                             index_move_greedy=ConfigMCTS.index_move_greedy,
                             exploration_constant=ConfigMCTS.exploration_constant,
                             filters=ConfigModel.filters, depth=ConfigModel.depth,
                             value_hidden=ConfigModel.value_hidden, bn_epsilon=ConfigModel.bn_epsilon,
                             cache_log2=ConfigSelfPlay.chess_cache_log2)
        eng.weights_key = None
        _CHESS_ENGINES.clear()
        _CHESS_ENGINES[key] = eng
    if not synthetic:
        wkey = model.content_hash if hasattr(model, "content_hash") else (id(model), getattr(model, "_version", None))
        if eng.weights_key != wkey:
            eng.set_weights(model.engine_weights())
            eng.weights_key = wkey
    return eng


def play_chess(model, n_games: int, base_seed: int, first_game: int = 0, sims: Optional[int] = None):
    """Batched chess self-play (BASELINE configs[4]).  Returns (states
    [M,8,8,118] f32 -- Board.full_state of each MCTS.play parent board, exact
    in f32 --, policies [M,1880] f64, rewards [M], records), in game order."""
    from custom_alphazero.chess import kernels as K
    from custom_alphazero.chess.board import Board as ChessBoard
    sims = int(sims or ConfigSelfPlay.mcts_iterations)
    eng = _chess_engine(model, min(n_games, ConfigSelfPlay.chess_concurrent_games), sims)
    eng.selfplay_run(first_game, n_games, base_seed)
    r = eng.selfplay_results()
    start = ChessBoard()._pos  # host bookkeeping only: FEN -> az_chess_pos
    states, policies, rewards, records = [], [], [], []
    for g in range(n_games):
        T = int(r["lengths"][g])
        pos = r["positions"][g, :T]
        # the reference's history deque: [0 x 7, state] on Board(), then
        # [0 x 6, start state, state] (chess/board.py docstring)
        hist = np.zeros((T, K.HISTORY), K.POS_DTYPE)
        valid = np.zeros((T, K.HISTORY), np.uint8)
        hist[:, 7], valid[:, 7] = pos, 1
        hist[1:, 6], valid[1:, 6] = start, 1
        states.append(K.encode(hist, valid) if T else np.zeros((0, 8, 8, K.PLANES), np.float32))
        pol = np.zeros((T, K.ACTIONS), np.float64)
        for t in range(T):
            n = int(r["policy_n"][g, t])
            pol[t, r["policy_actions"][g, t, :n]] = r["policy_probs"][g, t, :n]
        policies.append(pol)
        rewards.append(alternating_rewards(int(r["results"][g]), T))
        records.append(GameRecord(first_game + g, (base_seed + first_game + g) % 2 ** 32, T,
                                  int(r["results"][g]), int(r["expansions"][g]),
                                  r["moves"][g, :T].astype(np.int32)))
    return np.concatenate(states), np.vstack(policies), np.concatenate(rewards), records


def play(run_id: str, plays_inferences: Optional[Dict[str, Tuple[np.ndarray, float]]] = None,
         model=None, n_games: Optional[int] = None, base_seed: Optional[int] = None,
         first_game: int = 0, sims: Optional[int] = None):
    """Batched self-play.  Returns (states [M,H,W,4] f32, policies [M,A] f64,
    rewards [M] int64, records) concatenated in game order like the reference
    (self_play.py:112-118); with ConfigGeneral.game == "chess" the chess
    engine's (play_chess)."""
    if model is None:
        model = best_saved_model(run_id)
    n_games = int(n_games or ConfigSelfPlay.games_per_call)
    if base_seed is None:
        base_seed = ConfigSelfPlay.base_seed
    if base_seed is None:
        base_seed = int(time.time()) % (2 ** 32 - 1)
    if ConfigGeneral.game == "chess":
        return play_chess(model, n_games, base_seed, first_game)
    eng = _batched_engine(model, min(n_games, ConfigSelfPlay.concurrent_games), sims)
    if ConfigSelfPlay.cache_log2 and (plays_inferences is None
                                      or plays_inferences is not _CACHE_OWNER["dict"]):
        eng.cache_clear()
        _CACHE_OWNER["dict"] = plays_inferences
    eng.selfplay_run(first_game, n_games, base_seed)
    r = eng.selfplay_results()
    states, policies, rewards, records = [], [], [], []
    for g in range(n_games):
        T = int(r["lengths"][g])
        b = r["boards"][g, :T]
        s = np.zeros(b.shape + (4,), np.float32)
        s[..., 0] = b == 0
        s[..., 1] = b == 1
        s[..., 2] = b == -1
        s[..., 3] = 1.0
        states.append(s)
        policies.append(r["policies"][g, :T])
        rewards.append(alternating_rewards(int(r["results"][g]), T))
        records.append(GameRecord(first_game + g, (base_seed + first_game + g) % 2 ** 32, T,
                                  int(r["results"][g]), int(r["expansions"][g]),
                                  r["moves"][g, :T].copy()))
    return np.vstack(states), np.vstack(policies), np.concatenate(rewards), records


def exclude_null_games(states, policies, rewards):
    """self_play.py:155-162: drop samples of drawn games (reward 0)."""
    keep = rewards != 0
    return states[keep], policies[keep], rewards[keep]


def queue_payload(states, policies, values) -> dict:
    """The append_queue request body (serving/factory.py:69-80; schema
    ModelAppendQueueInputs, serving/schemas/schemas.py:27-30)."""
    return {"states": np.asarray(states).tolist(), "policies": np.asarray(policies).tolist(),
            "values": np.asarray(values).tolist()}


def write_queue_payload(path: str, states, policies, values) -> str:
    """File sink for the queue payload (the HTTP control plane is out of scope)."""
    with open(path, "w") as fp:
        json.dump(queue_payload(states, policies, values), fp)
    return path


def run(run_id: str, iterations: int = 1, queue_sink=None, model_loader=None):
    """self_play.__main__'s loop (self_play.py:128-185) without the HTTP
    control plane: poll the best model's hash (utils.best_saved_model_hash),
    reset plays_inferences when it changes, play a batch, drop draws
    (ConfigSelfPlay.exclude_null_games), checkpoint samples.npz every
    samples_checkpoint_frequency iterations, and hand the append_queue payload
    to `queue_sink` (a callable, e.g. list.append or an HTTP client).
    Returns the per-iteration sample counts."""
    from custom_alphazero.utils import best_saved_model_hash, reset_plays_inferences_dict
    load = model_loader or best_saved_model
    previous_hash, plays_inferences, model, counts = object(), None, None, []
    for it in range(iterations):
        current = best_saved_model_hash(run_id)
        if current != previous_hash or model is None:
            plays_inferences = reset_plays_inferences_dict()
            model = load(run_id)
            previous_hash = current
        states, policies, rewards, _records = play(run_id, plays_inferences, model=model)
        if ConfigSelfPlay.exclude_null_games:
            states, policies, rewards = exclude_null_games(states, policies, rewards)
        if (it + 1) % ConfigSelfPlay.samples_checkpoint_frequency == 0:
            save_samples(run_id, it, states, policies, rewards)
        if queue_sink is not None:
            queue_sink(queue_payload(states, policies, rewards))
        counts.append(len(states))
    return counts


def save_samples(run_id: str, iteration: int, states, policies, rewards) -> str:
    """samples.npz with keys states/policies/values (self_play.py:170-178,
    paths.py:37-40 layout results/{game}/{run_id}/self_play/iteration_k/)."""
    path = os.path.join(ConfigPath.results_dir, ConfigGeneral.game, run_id,
                        ConfigPath.self_play_dir, f"iteration_{iteration}")
    os.makedirs(path, exist_ok=True)
    out = os.path.join(path, ConfigPath.samples_file)
    np.savez(out, states=states, policies=policies, values=rewards)
    return out
