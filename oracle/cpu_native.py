"""ctypes binding of oracle/az_cpu.c, the native CPU self-play engine
(TEST INFRASTRUCTURE: bench.py's cpu_baseline_native leg and tests/ only).

fold_for_cpu() folds BatchNorm into the convs (float64, like the engine's
host folding) and flattens the weights in az_cpu.c's order."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def _cpu_flags():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    return set(line.split(":", 1)[1].split())
    except OSError:
        pass
    return set()


def load():
    global _lib
    if _lib is None:
        v4 = {"avx512f", "avx512bw", "avx512dq", "avx512vl"} <= _cpu_flags()
        _lib = ctypes.CDLL(os.path.join(_HERE, "_build", "libazcpu_v4.so" if v4 else "libazcpu_v3.so"))
        _lib.azc_selfplay.restype = ctypes.c_int
        _lib.azc_selfplay.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                                                          ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        _lib.azc_forward_probe.restype = ctypes.c_int
        _lib.azc_forward_probe.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 4
        _lib.azc_weight_count.restype = ctypes.c_int64
        _lib.azc_weight_count.argtypes = [ctypes.c_int] * 5
    return _lib


def _fold(w, unit, eps):
    k = np.asarray(w[unit + ".kernel"], np.float64)
    b = np.asarray(w[unit + ".bias"], np.float64)
    g, beta, m, v = (np.asarray(w[f"{unit}.{f}"], np.float64) for f in ("gamma", "beta", "mean", "var"))
    sc = g / np.sqrt(v + eps)
    return k * sc, (b - m) * sc + beta


def fold_for_cpu(w, H, W, A, depth, hidden=256, eps=1e-3):
    parts = []
    k, b = _fold(w, "stem", eps)
    parts += [k.reshape(9, -1, 128), b]
    for d in range(depth):
        for u in ("conv1", "conv2"):
            k, b = _fold(w, f"block{d}.{u}", eps)
            parts += [k.reshape(9, 128, 128), b]
        k, b = _fold(w, f"block{d}.res", eps)
        parts += [k.reshape(128, 128), b]
    k, b = _fold(w, "policy.conv", eps)
    parts += [k.reshape(128, 2), b]
    k, b = _fold(w, "value.conv", eps)
    parts += [k.reshape(128), b]
    parts += [np.asarray(w["policy.dense.kernel"]), np.asarray(w["policy.dense.bias"]),
              np.asarray(w["value.dense1.kernel"]), np.asarray(w["value.dense1.bias"]),
              np.asarray(w["value.dense2.kernel"]).reshape(-1), np.asarray(w["value.dense2.bias"])]
    flat = np.concatenate([np.asarray(p, np.float64).reshape(-1) for p in parts]).astype(np.float32)
    assert flat.size == load().azc_weight_count(H, W, A, depth, hidden), flat.size
    return flat


def forward(flat, board, gravity, depth, hidden=256):
    H, W = board.shape
    A = W if gravity else H * W
    probs = np.zeros(A, np.float32)
    value = np.zeros(1, np.float32)
    b = np.ascontiguousarray(board, np.int8)
    rc = load().azc_forward_probe(H, W, int(gravity), depth, hidden, flat.ctypes.data, b.ctypes.data,
                                  probs.ctypes.data, value.ctypes.data)
    assert rc == 0
    return probs, float(value[0])


def selfplay(flat, H, W, n, gravity, sims, depth, threads, seconds, seed0=40_000_000, cache_log2=22, hidden=256):
    out = np.zeros(6, np.float64)
    rc = load().azc_selfplay(H, W, n, int(gravity), sims, depth, hidden, flat.ctypes.data, threads,
                             float(seconds), seed0, cache_log2, out.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"azc_selfplay failed ({rc})")
    games, exps, evals, plies, hits, wall = out.tolist()
    return {"games": int(games), "expansions": int(exps), "evaluations": int(evals), "plies": int(plies),
            "cache_hits": int(hits), "seconds": wall}
