"""Helpers on the self-play path (reference custom_alphazero/utils.py:24-133)."""
import json
import os
from typing import Optional, Union

from custom_alphazero.config import ConfigConnectN, ConfigGeneral, ConfigPath
from custom_alphazero.connect_n.board import Board


def set_gpu_index(gpu_index: Union[int, str]):
    os.environ["CUDA_VISIBLE_DEVICES"] = str(gpu_index)


def reset_plays_inferences_dict() -> dict:
    """The reference returns a Manager().dict() shared by its worker processes
    (utils.py:38-39).  Here the cache lives on the device (self_play.play):
    the returned dict is a token -- passing the same object to play() keeps
    the device cache, a new one empties it."""
    return {}


def get_all_possible_moves():
    if ConfigGeneral.game == "chess":  # utils.py:13-15
        from custom_alphazero.chess.utils import get_all_possible_moves as chess_moves
        return chess_moves()
    return Board.get_all_possible_moves()


def input_dim():
    """Board().full_state.shape of the configured game: (H, W, 4), or chess's
    (8, 8, 118) (chess/board.py:55-73; static, no device call)."""
    if ConfigGeneral.game == "chess":
        return (8, 8, 118)
    return Board().full_state.shape


def init_model(path: Optional[str] = None, seed: Optional[int] = None):
    from custom_alphazero.model.policy_value import PolicyValueModel
    model = PolicyValueModel(input_dim=input_dim(),
                             action_space=len(get_all_possible_moves()), seed=seed)
    if path is not None:
        model.load_with_meta(path)
    return model


def _evaluation_path(run_id: str) -> str:
    return os.path.join(ConfigPath.results_dir, ConfigGeneral.game, run_id,
                        ConfigPath.evaluation_dir)


def last_evaluation_iteration_name(evaluation_path: str, prefix: str = "iteration",
                                   sep: str = "_") -> Optional[str]:
    if not os.path.exists(evaluation_path):
        return None
    done = [d for d in os.listdir(evaluation_path)
            if d.startswith(prefix)
            and os.path.exists(os.path.join(evaluation_path, d, ConfigPath.model_success))]
    return max(done, key=lambda d: int(d.split(sep)[-1])) if done else None


def best_saved_model(run_id: str):
    path = _evaluation_path(run_id)
    name = last_evaluation_iteration_name(path)
    if name is None:
        print(f"Warning: no model found at {path}, initializing best model with random weights")
        return init_model()
    return init_model(os.path.join(path, name))


def best_saved_model_hash(run_id: str) -> Optional[str]:
    path = _evaluation_path(run_id)
    name = last_evaluation_iteration_name(path)
    if name is None:
        return None
    meta = os.path.join(path, name, ConfigPath.model_meta)
    if not os.path.exists(meta):
        return None
    with open(meta) as fp:
        return json.load(fp).get("hash")


def board_shape():
    return ConfigConnectN.board_height, ConfigConnectN.board_width
