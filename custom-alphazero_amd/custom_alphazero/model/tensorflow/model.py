"""Import-path compatibility: the reference's callers import the model from
custom_alphazero.model.tensorflow.model (mcts/mcts.py:9, utils.py:10).  The
implementation is model/policy_value.py (PyTorch-held weights, libaz forward);
no TensorFlow is involved."""
from custom_alphazero.model.policy_value import PolicyValueModel  # noqa: F401
