"""Synthetic, exactly-representable board evaluator (TEST INFRASTRUCTURE).

This module is part of the oracle: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it.

Why it exists: the reference's MCTS (custom_alphazero/mcts/mcts.py:122-143)
asks a model for ``(probabilities[A] f32, value f32)`` per leaf board.  To pin
the tree arithmetic bit-for-bit against the *real* reference, the golden
generator (tests/golden/make_golden.py) runs the reference with a stub model
that returns this function's outputs, and the GPU engine has the same function
compiled in (``AZ_EVAL_SYNTHETIC`` in custom-alphazero_amd/csrc/az_common.h).
Every output is a dyadic rational (k/64 priors, k/128 values), so f32
representation is exact on every side and only the reference's own arithmetic
(f32 normalisation, f64 UCB, f64 backup) is being compared.

Board encoding: the canonical board (side to move = +1, reference
connect_n/board.py:244-246) as two bit masks ``own`` (cells == +1) and ``opp``
(cells == -1), bit index ``y * W + x`` (row 0 = top row, as the reference's
``array``).  Masks may exceed 64 bits (9x9 = 81 cells).
"""

M64 = (1 << 64) - 1


def splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def board_hash(own: int, opp: int) -> int:
    h = splitmix64(own & M64)
    h = splitmix64(h ^ ((own >> 64) & M64))
    h = splitmix64(h ^ (opp & M64))
    h = splitmix64(h ^ ((opp >> 64) & M64))
    return h


def synth_eval(own: int, opp: int, action_space: int):
    """Return (probs: list[float] of length A, value: float); all exact in f32.

    probs[a] = (5-bit field + 1) / 64, 12 fields per 64-bit word, re-mixed
    every 12 actions.  One board in 64 returns all-zero probabilities to
    exercise the reference's zero-sum branch (mcts/utils.py:8-9), which
    yields float64 uniform priors.  value = (top byte - 128) / 128.
    """
    h = board_hash(own, opp)
    vh = splitmix64(h ^ 0x5555555555555555)
    value = ((vh >> 56) - 128) / 128.0
    if (vh & 0x3F) == 0:
        return [0.0] * action_space, value
    probs = []
    word = h
    for a in range(action_space):
        if a and a % 12 == 0:
            word = splitmix64(word)
        probs.append((((word >> (5 * (a % 12))) & 31) + 1) / 64.0)
    return probs, value


def masks_from_array(array, width: int):
    """(own, opp) masks from a canonical int8 [H, W] array-like."""
    own = opp = 0
    for y, row in enumerate(array):
        for x, cell in enumerate(row):
            if cell == 1:
                own |= 1 << (y * width + x)
            elif cell == -1:
                opp |= 1 << (y * width + x)
    return own, opp


def masks_from_full_state(state):
    """(own, opp) masks from a full_state [H, W, 4] (channels empty/own/opp/turn)."""
    height = len(state)
    width = len(state[0])
    own = opp = 0
    for y in range(height):
        for x in range(width):
            if state[y][x][1] == 1.0:
                own |= 1 << (y * width + x)
            elif state[y][x][2] == 1.0:
                opp |= 1 << (y * width + x)
    return own, opp
