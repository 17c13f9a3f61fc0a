"""Connect-N board with the reference API (connect_n/board.py:12-271).

Host-side convenience object: the search never touches it (libaz keeps boards
as bit masks on the device, csrc/az_device.h).  Semantics the device must
agree with -- canonical mirroring under keep_same_player, Board.moves order,
the action order of get_all_possible_moves -- are pinned by
tests/test_api_cpu.py against the reference's own outputs.
"""
import hashlib
from copy import deepcopy
from itertools import product
from typing import List, Optional

import numpy as np

from custom_alphazero.config import ConfigConnectN
from custom_alphazero.connect_n.move import Move


def _dims():
    c = ConfigConnectN
    return c.board_height, c.board_width


class Board:
    def __init__(self, array: Optional[np.ndarray] = None):
        c = ConfigConnectN
        if not 2 <= c.n <= min(c.board_width, c.board_height):
            raise AssertionError("n must fit on the board")
        self.board_width, self.board_height = c.board_width, c.board_height
        self.n, self.gravity = c.n, c.gravity
        self.black, self.empty, self.white = c.black, c.empty, c.white
        self.pieces = dict(c.pieces)
        self.pieces_to_int = {sym: val for val, sym in self.pieces.items()}
        self.played_moves: List[Move] = []
        if array is None:
            self.array = np.zeros((self.board_height, self.board_width), np.int8)
        else:
            if not isinstance(array, np.ndarray):
                raise AssertionError("array must be an np.ndarray")
            if array.shape != (self.board_height, self.board_width):
                raise AssertionError("array shape does not match the board")
            if np.unique(array).size > len(self.pieces):
                raise AssertionError("unknown pieces")
            self.array = array.astype(np.int8)
        self.turn = self.white
        self.fullmove_number = 0
        self.game_over = False
        self.is_null = None

    # ------------------------------------------------------------ identity
    def __repr__(self):
        return "\n".join("".join(self.pieces[int(v)] for v in row) for row in self.array)

    def __hash__(self):
        return int(hashlib.md5(repr(self).encode("utf-8")).hexdigest(), 16)

    def __eq__(self, other: "Board"):
        return np.array_equal(self.array, other.array)

    def repr_graphviz(self) -> str:
        return "\n".join("".join(" . " if self.pieces[int(v)] == "." else self.pieces[int(v)]
                                 for v in row) for row in self.array)

    def repr_list_played_moves(self) -> str:
        if not self.gravity:
            raise NotImplementedError
        return "".join(str(m.x + 1) for m in self.played_moves)

    def display_ascii(self):
        print(repr(self))

    # ------------------------------------------------------------ encodings
    @property
    def turn_mirror(self) -> int:
        return self.black if self.turn == self.white else self.white

    @property
    def array_one_hot(self) -> np.ndarray:
        return np.eye(len(self.pieces))[self.array]

    @property
    def array_one_hot_mirror(self) -> np.ndarray:
        return np.eye(len(self.pieces))[self.mirror()]

    def _state(self, one_hot, turn):
        plane = np.full(self.array.shape + (1,), float(turn))
        return np.concatenate([one_hot, plane], axis=-1).astype(np.float32)

    @property
    def full_state(self) -> np.ndarray:
        return self._state(self.array_one_hot, self.turn)

    @property
    def full_state_mirror(self) -> np.ndarray:
        return self._state(self.array_one_hot_mirror, self.turn_mirror)

    @staticmethod
    def from_one_hot(array_oh: np.ndarray) -> np.ndarray:
        idx = np.argmax(array_oh, axis=-1)
        idx[idx > (len(ConfigConnectN.pieces) - 1) / 2] = -1
        return idx

    def mirror(self) -> np.ndarray:
        return -self.array

    # ------------------------------------------------------------ moves
    @property
    def odd_moves_number(self) -> bool:
        return bool(self.fullmove_number % 2)

    @property
    def moves(self) -> List[Move]:
        free = self.array == self.empty
        if self.gravity:
            return [Move(True, int(x)) for x in np.flatnonzero(free[0])]
        ys, xs = np.nonzero(free)  # row-major scan, as np.where
        return [Move(False, int(x), int(y)) for y, x in zip(ys, xs)]

    def last_move(self) -> Optional[Move]:
        return self.played_moves[-1] if self.played_moves else None

    @staticmethod
    def get_all_possible_moves() -> List[Move]:
        c = ConfigConnectN
        if c.gravity:
            return [Move(True, x) for x in range(c.board_width)]
        return [Move(False, x, y) for x, y in product(range(c.board_width), range(c.board_height))]

    def legal_moves_mask(self, all_possible_moves: List[Move]) -> np.ndarray:
        legal = set(m.key() for m in self.moves)
        return np.asarray([m.key() in legal for m in all_possible_moves])

    def get_random_move(self) -> Optional[Move]:
        options = self.moves
        if not options:
            return None
        return np.random.choice(options)

    # ------------------------------------------------------------ rules
    def is_game_over(self) -> bool:
        return self.game_over

    def update_array(self):
        pass

    def _line_length(self, y0, x0, dy, dx):
        stone = self.array[y0, x0]
        run, y, x = 0, y0 + dy, x0 + dx
        while 0 <= y < self.board_height and 0 <= x < self.board_width and self.array[y, x] == stone:
            run += 1
            y, x = y + dy, x + dx
        return run

    def update_game_over(self, last_move_x: int, last_move_y: int):
        if self.game_over:
            return
        for dx, dy in ConfigConnectN.directions:
            total = 1 + self._line_length(last_move_y, last_move_x, dy, dx) \
                + self._line_length(last_move_y, last_move_x, -dy, -dx)
            if total >= ConfigConnectN.n:
                self.game_over, self.is_null = True, False
                return
        if not self.moves:
            self.game_over, self.is_null = True, True

    def push(self, move: Move):
        if self.gravity:
            column = self.array[:, move.x]
            empty_rows = np.flatnonzero(column == self.empty)
            if empty_rows.size == 0:
                raise AssertionError("column is full")
            # the stone falls to the row just above the first occupied cell
            occupied = np.flatnonzero(column != self.empty)
            row = (occupied[0] - 1) if occupied.size else self.board_height - 1
            if row < 0 or column[row] != self.empty:
                raise AssertionError("illegal move")
            self.array[row, move.x] = self.turn
            self.update_game_over(move.x, int(row))
        else:
            if self.array[move.y, move.x] != self.empty:
                raise AssertionError("cell is occupied")
            self.array[move.y, move.x] = self.turn
            self.update_game_over(move.x, move.y)
        self.turn = self.turn_mirror

    def play(self, move: Optional[Move], on_copy: bool = False,
             keep_same_player: bool = False) -> "Board":
        if move is None or self.game_over:
            return self
        target = deepcopy(self) if on_copy else self
        target.push(move)
        target.fullmove_number += 1
        if keep_same_player:
            target.array = target.mirror()
            target.turn = self.white
        target.played_moves.append(move)
        return target

    def play_random(self, on_copy: bool = False, keep_same_player: bool = False) -> "Board":
        return self.play(self.get_random_move(), on_copy, keep_same_player)

    def get_result(self, keep_same_player: bool = False):
        if self.is_null is None or not self.game_over:
            return None
        if self.is_null:
            return 0
        if keep_same_player:
            return self.white
        return self.white if self.odd_moves_number else self.black
