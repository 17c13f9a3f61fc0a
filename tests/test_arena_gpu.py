"""Arena (reference evaluation/evaluate.py:29-134) on the device: the batched
evaluation (all games at once, one engine per model) reproduces the
reference's sequential game loop game by game."""
import numpy as np
import pytest

from custom_alphazero.config import ConfigSelfPlay, ConfigServing
from custom_alphazero.connect_n.board import Board
from custom_alphazero.evaluation import evaluate
from custom_alphazero.model.tensorflow.model import PolicyValueModel

pytestmark = pytest.mark.gpu


@pytest.fixture
def two_models(monkeypatch):
    monkeypatch.setattr(ConfigSelfPlay, "mcts_iterations", 12)
    shape = Board().full_state.shape
    a = PolicyValueModel(input_dim=shape, action_space=7, seed=1)
    b = PolicyValueModel(input_dim=shape, action_space=7, seed=2)
    return a, b


@pytest.mark.parametrize("with_mcts", [False, True])
@pytest.mark.parametrize("deterministic", [True, False])
def test_batched_arena_matches_sequential(two_models, with_mcts, deterministic):
    a, b = two_models
    n = 4
    tb, ts = [], []
    _, batched = evaluate.evaluate_two_models_batched(a, b, n_games=n, evaluate_with_mcts=with_mcts,
                                                      deterministic=deterministic, seed=7, trace=tb)
    moves = Board.get_all_possible_moves()
    seq = [evaluate._single_game_evaluation(a, b, g, moves, with_mcts, False, deterministic,
                                            rng=np.random.RandomState(7 + g), trace=ts)[0]
           for g in range(n)]
    assert batched == seq
    for x, y in zip(tb, ts):  # same final positions, move for move
        np.testing.assert_array_equal(x, y)
    assert set(batched) <= {-1, 0, 1}


def test_evaluate_two_models_score(two_models, monkeypatch):
    a, b = two_models
    monkeypatch.setattr(ConfigServing, "evaluation_games_number", 2)
    score, solver = evaluate.evaluate_two_models(a, b, deterministic=True)
    assert 0.0 <= score <= 1.0 and solver is None
    with pytest.raises(NotImplementedError):
        evaluate.evaluate_two_models(a, b, evaluate_with_solver=True)
