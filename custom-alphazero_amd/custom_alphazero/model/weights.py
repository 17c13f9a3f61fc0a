"""Weight layout of the policy/value network and its Keras-default init.

Names follow the reference's layer structure (model/tensorflow/model.py:21-188,
base_layers.py:20-125): every InnerConvBlock is a unit with
kernel[kh][kw][cin][cout], bias, gamma, beta, mean, var (BatchNormalization
moving statistics); Dense layers have kernel[in][out] and bias.
Initialisation mirrors tf.keras defaults: glorot-uniform kernels, zero
biases, BN gamma 1 / beta 0 / mean 0 / var 1 (un-vendored TF 2.7.1 defaults,
SURVEY.md section 3.4).  Random streams come from torch.Generator(seed).
"""
import math

import numpy as np

BN_FIELDS = ("gamma", "beta", "mean", "var")


def conv_units(depth):
    units = [("stem", 3, None)]
    for d in range(depth):
        units += [(f"block{d}.conv1", 3, None), (f"block{d}.conv2", 3, None),
                  (f"block{d}.res", 1, None)]
    return units


def weight_spec(height, width, action_space, filters=128, depth=4, hidden=256, in_channels=4):
    """Ordered list of (name, shape)."""
    F, HW = filters, height * width
    spec = []

    def unit(name, k, cin, cout):
        spec.append((name + ".kernel", (k, k, cin, cout)))
        spec.append((name + ".bias", (cout,)))
        for f in BN_FIELDS:
            spec.append((f"{name}.{f}", (cout,)))

    unit("stem", 3, in_channels, F)
    for d in range(depth):
        unit(f"block{d}.conv1", 3, F, F)
        unit(f"block{d}.conv2", 3, F, F)
        unit(f"block{d}.res", 1, F, F)
    unit("policy.conv", 1, F, 2)
    spec.append(("policy.dense.kernel", (2 * HW, action_space)))
    spec.append(("policy.dense.bias", (action_space,)))
    unit("value.conv", 1, F, 1)
    spec.append(("value.dense1.kernel", (HW, hidden)))
    spec.append(("value.dense1.bias", (hidden,)))
    spec.append(("value.dense2.kernel", (hidden, 1)))
    spec.append(("value.dense2.bias", (1,)))
    return spec


def keras_order(spec):
    """Names of `spec` in the order tf.keras `Model.get_weights()` returns
    them for the reference's PolicyValueModel (model/tensorflow/model.py:
    152-170; un-vendored TF 2.7.1, parity unpinned): per top-level layer
    (residual tower, policy head, value head, in attribute order), that
    layer's trainable weights depth-first (conv kernel, bias, BN gamma, beta
    per InnerConvBlock; Dense kernel, bias), then its non-trainable ones (BN
    moving mean, variance) depth-first."""
    names = [n for n, _ in spec]

    def split(prefixes):
        own = [n for n in names if n.split(".")[0] in prefixes]
        train = [n for n in own if n.rsplit(".", 1)[1] not in ("mean", "var")]
        return train + [n for n in own if n.rsplit(".", 1)[1] in ("mean", "var")]

    tower = {"stem"} | {n.split(".")[0] for n in names if n.startswith("block")}
    out = split(tower) + split({"policy"}) + split({"value"})
    assert sorted(out) == sorted(names)
    return out


def reference_hash(arrays):
    """The reference's weight hash (model/tensorflow/model.py:172-177): the
    sum over get_weights() of md5(str(weight)).  str() is numpy's summarised
    print form (arrays over 1000 elements show only their corners), so two
    weight sets that differ only inside large arrays hash the same; use
    content_hash to detect a change of weights."""
    import hashlib
    return sum(int(hashlib.md5(str(np.asarray(w, np.float32)).encode("utf-8")).hexdigest(), 16)
               for w in arrays)


def content_hash(arrays):
    """md5 over the raw float32 bytes of every array (order-sensitive)."""
    import hashlib
    h = hashlib.md5()
    for w in arrays:
        h.update(np.ascontiguousarray(w, np.float32).tobytes())
    return h.hexdigest()


def glorot_limit(shape):
    if len(shape) == 4:
        rf = shape[0] * shape[1]
        fan_in, fan_out = rf * shape[2], rf * shape[3]
    else:
        fan_in, fan_out = shape[0], shape[1]
    return math.sqrt(6.0 / (fan_in + fan_out))


def init_weights(spec, seed=0, randomize_bn=False):
    """Keras-default init as float32 numpy arrays (dict name -> array).

    randomize_bn=True draws non-trivial BN statistics and biases so tests
    exercise the folding (a fresh Keras model has identity BN).
    """
    import torch

    gen = torch.Generator(device="cpu").manual_seed(int(seed))
    out = {}
    for name, shape in spec:
        field = name.rsplit(".", 1)[1]
        if field == "kernel":
            lim = glorot_limit(shape)
            t = (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1) * lim
        elif randomize_bn and field in ("bias", "beta", "mean"):
            t = (torch.rand(shape, generator=gen, dtype=torch.float64) - 0.5) * 0.2
        elif randomize_bn and field == "gamma":
            t = 0.8 + 0.4 * torch.rand(shape, generator=gen, dtype=torch.float64)
        elif randomize_bn and field == "var":
            t = 0.5 + torch.rand(shape, generator=gen, dtype=torch.float64)
        elif field in ("gamma", "var"):
            t = torch.ones(shape, dtype=torch.float64)
        else:
            t = torch.zeros(shape, dtype=torch.float64)
        out[name] = t.to(torch.float32).numpy()
    return out


def as_list(weights, spec):
    return [np.asarray(weights[name], np.float32).reshape(shape) for name, shape in spec]
