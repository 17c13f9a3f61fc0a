"""MI355X-native drop-in for custom_alphazero's self-play path.

Same import paths as the reference (custom_alphazero.mcts.mcts.MCTS,
custom_alphazero.self_play.play_game, custom_alphazero.model.tensorflow.model.
PolicyValueModel, custom_alphazero.connect_n.board.Board, custom_alphazero.config);
the search and the network run in libaz (HIP, gfx950) through ctypes.
"""
import os as _os
import sys as _sys

__all__ = ["config", "engine"]

# HIP hardware queues per process (GPU_MAX_HW_QUEUES, read once when HIP
# initialises).  HIP's default of 4 makes a third self-play lane's stream share
# a queue (-27%); with 8 the engine's auto rule runs 1536-4096 slots on 3 lanes
# (+4.9% games/s at configs[1]) -- the configuration
# bench.py measures.  Raised to 8 here, at import, as bench.py does, unless
# this process has already initialised HIP through torch (HIP then keeps the
# count it made, and the variable is left as it is) or AZ_KEEP_HW_QUEUES=1
# asks to keep the caller's value.  libaz reads the variable when it loads.
HW_QUEUES_DEFAULT = 8


def _default_hw_queues():
    if _os.environ.get("AZ_KEEP_HW_QUEUES") == "1":
        return
    try:
        cur = int(_os.environ.get("GPU_MAX_HW_QUEUES", "") or 4)
    except ValueError:
        cur = 4
    if cur >= HW_QUEUES_DEFAULT:
        return
    torch = _sys.modules.get("torch")
    cuda = getattr(torch, "cuda", None) if torch is not None else None
    if cuda is not None and cuda.is_initialized():
        return
    _os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES_DEFAULT)


_default_hw_queues()
