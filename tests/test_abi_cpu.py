"""CPU checks of the drop-in boundary: libaz loads and exports every symbol
include/*.h declares (az.h, az_chess.h); the ctypes structs match the header layout."""
import ctypes
import os
import re

import numpy as np
import pytest

from custom_alphazero import engine as az

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    names = set()
    for h in sorted(os.listdir(os.path.join(REPO, "include"))):
        if h.endswith(".h"):
            src = open(os.path.join(REPO, "include", h)).read()
            names |= set(re.findall(r"^(?:int|const char\*)\s+(az_\w+)\(", src, re.M))
    return sorted(names)


def test_header_and_binding_agree():
    declared = header_functions()
    assert declared == sorted(az.EXPORTED)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(az.LIB_PATH):
        pytest.fail("libaz.so missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(az.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name
    L = az.load_library()
    assert L.az_abi_version() == 4


def test_struct_sizes_match_header():
    # az_config: 8 int32 + double + 4 int32 ... computed by hand from az.h
    assert ctypes.sizeof(az.Config) == 4 * 6 + 8 + 4 * 5 + 4 + 8 + 8 + 8 + 32
    assert ctypes.sizeof(az.Tensor) == 8 + 8 + 8 + 4 + 4
    assert ctypes.sizeof(az.Stats) == 8 * 8 + 8 + 8 * 7 + 8 * 7
    # az_chess_config: 2 int32, double, 6 int32, double, int64, int32 + 7 reserved
    assert ctypes.sizeof(az.ChessConfig) == 8 + 8 + 24 + 8 + 8 + 4 + 28


def test_engine_fails_loudly_without_gpu():
    """No CPU fallback: without a visible HIP device the engine refuses to
    start (the product path never routes through the oracle)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from custom_alphazero import engine as az
    with pytest.raises(az.AzError, match="no HIP device"):
        az.Engine(6, 7, 4, True, 10, slots=4, evaluator=az.EVAL_SYNTHETIC)


def test_chess_kernels_fail_loudly_without_gpu():
    """The chess board seam has no CPU fallback either."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from custom_alphazero.chess import kernels as K
    from custom_alphazero.chess.board import Board
    b = Board()  # construction is host bookkeeping only
    with pytest.raises(az.AzError, match="no HIP device"):
        b.moves
    with pytest.raises(az.AzError, match="no HIP device"):
        K.encode(np.zeros((1, 8), K.POS_DTYPE), np.ones((1, 8), np.uint8))
