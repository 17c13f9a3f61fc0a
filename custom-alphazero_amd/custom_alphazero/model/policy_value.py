"""PolicyValueModel with the reference's call signature
(custom_alphazero/model/tensorflow/model.py:152-218).

PyTorch-ROCm only *holds* the weights (float32 tensors on the GPU, Keras
layout, names from model/weights.py); the forward runs in libaz
(az_forward: the conv16 tower + heads, csrc/az_nn.hip, az_conv16.hip).  Calling the
model returns (probabilities [B, A], value [B, 1]) as torch CPU tensors, so
the reference's `.numpy()` idiom (mcts.py:134-137) works unchanged.
"""
import json
import os

import numpy as np

from custom_alphazero import engine as az
from custom_alphazero.config import ConfigConnectN, ConfigModel, ConfigPath
from custom_alphazero.model.tf_checkpoint import load_keras_weights, save_keras_weights
from custom_alphazero.model.weights import (content_hash, init_weights, keras_order, reference_hash,
                                            weight_spec)


class PolicyValueModel:
    def __init__(self, input_dim, action_space, seed=None, device=0):
        import torch

        self.input_dim = tuple(int(d) for d in input_dim)
        self.action_space = int(action_space)
        H, W, C = self.input_dim
        self.depth = ConfigModel.depth
        self.spec = weight_spec(H, W, self.action_space, ConfigModel.filters, self.depth,
                                ConfigModel.value_hidden, C)
        if seed is None:
            seed = int.from_bytes(os.urandom(4), "little")
        self.device = torch.device("cuda", device)
        self.weights = {k: torch.from_numpy(v).to(self.device)
                        for k, v in init_weights(self.spec, seed).items()}
        self.steps = 0
        self.learning_rate = ConfigModel.maximum_learning_rate
        self._engine = None
        self._engine_version = -1
        self._version = 0
        # the reference's constructor runs a dummy forward on
        # np.random.rand(1, *input_dim) (model/tensorflow/model.py:167-169):
        # the same draws from numpy's global stream, so a caller seeding
        # np.random before building the model (self_play.play_game) sees the
        # reference's stream afterwards
        np.random.rand(1, *self.input_dim)

    # ------------------------------------------------------------ weights
    def engine_weights(self):
        return [(name, self.weights[name]) for name, _ in self.spec]

    @property
    def weight_names(self):
        """get_weights()/set_weights() order: tf.keras's for the reference
        model (weights.keras_order)."""
        return keras_order(self.spec)

    def get_weights(self):
        shapes = dict(self.spec)
        return [self.weights[n].detach().cpu().numpy().reshape(shapes[n]) for n in self.weight_names]

    def set_weights(self, arrays):
        import torch
        arrays = list(arrays)
        if len(arrays) != len(self.spec):
            raise ValueError(f"expected {len(self.spec)} arrays, got {len(arrays)}")
        shapes = dict(self.spec)
        for name, a in zip(self.weight_names, arrays):
            a = np.asarray(a, np.float32)
            if a.shape != tuple(shapes[name]):
                raise ValueError(f"{name}: shape {a.shape} != {shapes[name]}")
            self.weights[name] = torch.from_numpy(a.copy()).to(self.device)
        self._version += 1

    @property
    def hash(self) -> int:
        """The reference's hash, sum of md5(str(weight)) over get_weights()
        (model.py:172-177): a meta.json the reference wrote validates here."""
        return reference_hash(self.get_weights())

    @property
    def content_hash(self) -> str:
        """md5 of the raw float32 weights: changes whenever any weight does
        (the reference hash only sees the corners of large arrays)."""
        return content_hash(self.get_weights())

    def is_equal(self, other: "PolicyValueModel"):
        return self.hash == other.hash

    # ------------------------------------------------------------ forward
    def _eng(self):
        if self._engine is None:
            H, W, C = self.input_dim
            if C == 118:  # chess planes (chess/board.py:55-73): the chess engine's forward
                self._engine = az.ChessEngine(1, slots=ConfigModel.forward_batch,
                                              evaluator=az.EVAL_NETWORK, filters=ConfigModel.filters,
                                              depth=self.depth, value_hidden=ConfigModel.value_hidden,
                                              bn_epsilon=ConfigModel.bn_epsilon,
                                              device=self.device.index or 0)
            else:
                c = ConfigConnectN
                self._engine = az.Engine(H, W, min(c.n, H, W), c.gravity, 1,
                                         slots=ConfigModel.forward_batch, evaluator=az.EVAL_NETWORK,
                                         filters=ConfigModel.filters, depth=self.depth,
                                         value_hidden=ConfigModel.value_hidden,
                                         bn_epsilon=ConfigModel.bn_epsilon,
                                         device=self.device.index or 0)
        if self._engine_version != self._version:
            self._engine.set_weights(self.engine_weights())
            self._engine_version = self._version
        return self._engine

    def __call__(self, inputs, training=False):
        import torch
        x = inputs.numpy() if hasattr(inputs, "numpy") else np.asarray(inputs)
        x = np.asarray(x, np.float32).reshape((-1,) + self.input_dim)
        probs, values = self._eng().forward(x)
        return torch.from_numpy(probs), torch.from_numpy(values.reshape(-1, 1))

    call = __call__

    # ------------------------------------------------------------ persistence
    def save_with_meta(self, path):
        os.makedirs(path, exist_ok=True)
        # the reference's files: Model.save_weights(path/model) in TensorFlow's
        # checkpoint format (model.py:203-204; model/tf_checkpoint.py)
        shapes = dict(self.spec)
        save_keras_weights(os.path.join(path, ConfigPath.model_prefix), self.spec,
                           {n: w.reshape(shapes[n]) for n, w in zip(self.weight_names, self.get_weights())})
        # `hash` is the reference's (sum of md5(str(w)), model.py:172-177): it
        # depends on numpy's str() of an array, so a checkpoint moved between
        # numpy versions may not reproduce it; `content_hash` (md5 of the raw
        # bytes) is recorded beside it and accepted on load
        meta = {"steps": int(self.steps), "learning_rate": float(self.learning_rate),
                "hash": self.hash, "content_hash": self.content_hash}
        with open(os.path.join(path, ConfigPath.model_meta), "w") as fp:
            json.dump(meta, fp, sort_keys=True, indent=4)
        open(os.path.join(path, ConfigPath.model_success), "wb").close()

    def load_with_meta(self, path):
        if not os.path.exists(os.path.join(path, ConfigPath.model_success)):
            raise AssertionError(f"No verification file of the model found at {path}!")
        prefix = os.path.join(path, ConfigPath.model_prefix)
        if os.path.exists(prefix + ".index"):  # Model.load_weights (model.py:194): a TF checkpoint
            w = load_keras_weights(prefix, self.spec)
            self.set_weights([w[name] for name in self.weight_names])
        else:  # the .npz this package's earlier builds wrote
            with np.load(prefix + ".npz", allow_pickle=False) as z:
                self.set_weights([z[name] for name in self.weight_names])
        with open(os.path.join(path, ConfigPath.model_meta)) as fp:
            meta = json.load(fp)
        self.steps = int(meta.get("steps", 0))
        self.learning_rate = float(meta.get("learning_rate", self.learning_rate))
        # the reference's hash (a meta.json the reference wrote), or the raw-bytes
        # hash this package records (also what its earlier builds stored as
        # `hash`): either identifies the weights
        content = self.content_hash
        if self.hash != meta.get("hash") and content not in (meta.get("content_hash"), meta.get("hash")):
            raise AssertionError(f"Unexpected weights hash recovered during model loading at {path}!")

    def get_learning_rate(self) -> float:
        return float(self.learning_rate)

    def update_learning_rate(self, learning_rate: float):
        self.learning_rate = float(learning_rate)
