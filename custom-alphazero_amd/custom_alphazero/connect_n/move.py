"""Connect-N move value object (API of reference connect_n/move.py:5-39)."""
from functools import total_ordering
from typing import Optional


@total_ordering
class Move:
    __slots__ = ("gravity", "x", "y")

    def __init__(self, gravity: bool, x: int, y: Optional[int] = None):
        if gravity and y is not None:
            raise AssertionError("a gravity move is a column only")
        if not gravity and y is None:
            raise AssertionError("a no-gravity move needs a row")
        self.gravity = gravity
        self.x = int(x)
        self.y = None if gravity else int(y)

    def key(self):
        return (self.x, self.y)

    def __eq__(self, other):
        return self.key() == (other.x, other.y)

    def __lt__(self, other):
        return self.key() < (other.x, other.y)

    def __hash__(self):
        return hash(self.key())

    def __str__(self):
        return str(self.x) if self.gravity else f"({self.x}, {self.y})"

    __repr__ = __str__
