"""Chess move value object, API of the reference's chess/move.py:8-69.

pos_from = (file, rank), pos_to = (file, rank, promotion letter or ""),
ordered as tuples (Move.__lt__, move.py:33-37): the order of
get_all_possible_moves.  `code` is libaz's uint16 encoding (include/az_chess.h:
from | to << 6 | promotion piece type << 12).
"""
from functools import total_ordering
from typing import Optional, Tuple

from custom_alphazero.config import ConfigChess

_PROMO_TYPE = {"": 0, "n": 2, "b": 3, "r": 4, "q": 5}
_PROMO_LETTER = {v: k for k, v in _PROMO_TYPE.items()}


@total_ordering
class Move:
    __slots__ = ("pos_from", "pos_to")

    def __init__(self, pos_from: Optional[Tuple[int, int]] = None,
                 pos_to: Optional[Tuple[int, int, str]] = None, uci: Optional[str] = None):
        if uci is not None:
            pos_from, pos_to = self.uci_to_coords(uci)
        assert pos_from is not None and pos_to is not None
        self.pos_from = tuple(pos_from)
        self.pos_to = tuple(pos_to)

    def __str__(self):
        return "({0}, {1}) -> ({2}, {3}, {4})".format(*self.pos_from, *self.pos_to)

    def __repr__(self):
        return str(self)

    def __eq__(self, other):
        return (self.pos_from, self.pos_to) == (other.pos_from, other.pos_to)

    def __lt__(self, other):
        return (self.pos_from, self.pos_to) < (other.pos_from, other.pos_to)

    def __hash__(self):
        return hash((self.pos_from, self.pos_to))

    @property
    def uci(self) -> str:
        return (chr(self.pos_from[0] + ord("a")) + str(self.pos_from[1] + 1)
                + chr(self.pos_to[0] + ord("a")) + str(self.pos_to[1] + 1) + self.pos_to[2])

    @staticmethod
    def uci_to_coords(uci: str):
        assert 4 <= len(uci) <= 5
        position_from = ord(uci[0]) - ord("a"), int(uci[1]) - 1
        position_to = ord(uci[2]) - ord("a"), int(uci[3]) - 1
        position_to = position_to + ((uci[4],) if len(uci) == 5 else ("",))
        return position_from, position_to

    @staticmethod
    def mirror(move: "Move") -> "Move":
        """The reference's Move.mirror (move.py:57-69): a point reflection of
        both squares (not python-chess's vertical flip); kept as is."""
        n = ConfigChess.board_size
        return Move(pos_from=(n - 1 - move.pos_from[0], n - 1 - move.pos_from[1]),
                    pos_to=(n - 1 - move.pos_to[0], n - 1 - move.pos_to[1], move.pos_to[2]))

    # ---------------------------------------------------------- libaz codes
    @property
    def code(self) -> int:
        f = self.pos_from[1] * 8 + self.pos_from[0]
        t = self.pos_to[1] * 8 + self.pos_to[0]
        return f | (t << 6) | (_PROMO_TYPE[self.pos_to[2]] << 12)

    @staticmethod
    def from_code(code: int) -> "Move":
        code = int(code)
        f, t, p = code & 63, (code >> 6) & 63, code >> 12
        return Move(pos_from=(f & 7, f >> 3), pos_to=(t & 7, t >> 3, _PROMO_LETTER[p]))
