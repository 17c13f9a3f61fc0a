"""normalize_probabilities with the reference's semantics (mcts/utils.py:4-16).

Host helper for API users; the device restates the same arithmetic
(csrc/az_device.h pairwise_sum_*).  numpy's float32 sum is pairwise; the
zero-sum branch returns a float64 uniform array.
"""
import numpy as np


def normalize_probabilities(probabilities: np.ndarray) -> np.ndarray:
    p = np.asarray(probabilities)
    if len(p) == 0:
        raise AssertionError("empty probability vector")
    total = p.sum()
    if total == 0:
        return np.full(len(p), 1.0 / len(p))
    return np.divide(p, total, out=np.zeros_like(p), where=total != 0)
