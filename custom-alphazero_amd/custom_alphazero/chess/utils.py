"""get_all_possible_moves (reference chess/utils.py:11-32): the 1880-move
action list, sorted by Move.__lt__; libaz derives it (az_chess_all_moves)."""
from functools import lru_cache
from typing import List

from custom_alphazero.chess import kernels as K
from custom_alphazero.chess.move import Move


@lru_cache(maxsize=1)
def _all_moves():
    return tuple(Move.from_code(c) for c in K.all_moves())


def get_all_possible_moves() -> List[Move]:
    return list(_all_moves())
