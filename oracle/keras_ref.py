"""Float64 numpy restatement of the reference's Keras forward (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module.  It restates, at inference (call(training=False)):
  ResidualTower  custom_alphazero/model/tensorflow/model.py:21-65
  PolicyHead     model.py:68-103 (conv1x1 -> BN -> ReLU -> Flatten -> Dense softmax)
  ValueHead      model.py:106-149 (conv1x1 -> BN -> ReLU -> Flatten -> Dense ReLU
                 -> Dense tanh)
  InnerConvBlock base_layers.py:20-66 (Conv2D 'same' + bias -> BN -> activation)
  OuterConvBlock base_layers.py:69-125 (two inner blocks + a 1x1 projection
                 residual with BN, Add, ReLU)
BatchNormalization uses moving statistics with tf.keras' default epsilon
1e-3.  TensorFlow 2.7.1 itself is not installed (no network), so this
restatement is pinned by its own fixtures only: "parity unpinned against TF"
(DESIGN.md).  Weight names: custom_alphazero/model/weights.py.
"""
import numpy as np


def conv2d_same(x, kernel, bias):
    """x [B,H,W,Cin], kernel [k,k,Cin,Cout] -> [B,H,W,Cout]; stride 1, SAME."""
    k = kernel.shape[0]
    p = k // 2
    B, H, W, _ = x.shape
    xp = np.pad(x, ((0, 0), (p, p), (p, p), (0, 0)))
    out = np.zeros((B, H, W, kernel.shape[3]), np.float64)
    for ky in range(k):
        for kx in range(k):
            out += xp[:, ky:ky + H, kx:kx + W, :] @ kernel[ky, kx]
    return out + bias


def batch_norm(x, w, unit, eps):
    g, b, m, v = (np.asarray(w[f"{unit}.{f}"], np.float64) for f in ("gamma", "beta", "mean", "var"))
    return (x - m) / np.sqrt(v + eps) * g + b


def inner(x, w, unit, eps, relu=True):
    y = conv2d_same(x, np.asarray(w[unit + ".kernel"], np.float64),
                    np.asarray(w[unit + ".bias"], np.float64))
    y = batch_norm(y, w, unit, eps)
    return np.maximum(y, 0.0) if relu else y


def forward(w, x, depth, eps=1e-3):
    """Returns (probs [B,A] float64, values [B] float64)."""
    x = np.asarray(x, np.float64)
    h = inner(x, w, "stem", eps)
    for d in range(depth):
        a = inner(h, w, f"block{d}.conv1", eps)
        a = inner(a, w, f"block{d}.conv2", eps, relu=False)
        r = inner(h, w, f"block{d}.res", eps, relu=False)
        h = np.maximum(a + r, 0.0)
    B = x.shape[0]
    p = inner(h, w, "policy.conv", eps).reshape(B, -1)  # Flatten on NHWC: (H, W, C)
    logits = p @ np.asarray(w["policy.dense.kernel"], np.float64) + np.asarray(w["policy.dense.bias"], np.float64)
    logits -= logits.max(axis=1, keepdims=True)
    e = np.exp(logits)
    probs = e / e.sum(axis=1, keepdims=True)
    v = inner(h, w, "value.conv", eps).reshape(B, -1)
    v = np.maximum(v @ np.asarray(w["value.dense1.kernel"], np.float64) + np.asarray(w["value.dense1.bias"], np.float64), 0.0)
    v = np.tanh(v @ np.asarray(w["value.dense2.kernel"], np.float64) + np.asarray(w["value.dense2.bias"], np.float64))
    return probs, v.reshape(B)
