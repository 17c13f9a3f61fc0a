"""Chess board with the reference API (custom_alphazero/chess/board.py:12-196).

The reference subclasses python-chess 1.9.4's Board.  Here the position is an
az_chess_pos record and every rules computation -- legal moves and their
order, the legal-move mask, outcome, push/mirror, full_state -- runs in
libaz's HIP kernels (include/az_chess.h, csrc/az_chess.h).  The host keeps
only bookkeeping: FEN text, the history deque and the move stack used by
is_repetition().

Behaviours kept from the reference as they are:
* play(keep_same_player=True) pushes, mirrors (python-chess mirror: vertical
  flip + colour swap) and sets turn = WHITE (board.py:162-173);
* python-chess's copy()/mirror() re-run the subclass __init__, so a copied or
  mirrored board starts from the start position's `array` and a history of
  [0 x 7, start-position state]; play() then appends the new state.  In MCTS
  use every non-root board therefore holds [0 x 6, start state, state];
* get_result() compares the result string's characters (board.py:181-193),
  so both "1-0" and "0-1" give 1 (a win for the side that just moved, in the
  canonical form) and "1/2-1/2" gives 0.
"""
from collections import deque
from typing import List, Optional

import numpy as np

from custom_alphazero.chess import kernels as K
from custom_alphazero.chess.move import Move
from custom_alphazero.config import ConfigChess

WHITE, BLACK = True, False
_SYMBOLS = "pnbrqk"
_RANK_1, _RANK_8 = 0xFF, 0xFF << 56
_FILE_A, _FILE_H = 0x0101010101010101, 0x8080808080808080
_ALL = (1 << 64) - 1


def _bit(sq):
    return 1 << sq


def _bswap(x):
    return int.from_bytes(int(x).to_bytes(8, "little"), "big")


def _clean_castling(p):
    """python-chess clean_castling_rights() (standard chess)."""
    pieces = [int(x) for x in p["pieces"]]
    co = [int(x) for x in p["occupied_co"]]
    c = int(p["castling_rights"]) & pieces[3]
    w = c & _RANK_1 & co[1] & (_bit(0) | _bit(7))
    b = c & _RANK_8 & co[0] & (_bit(56) | _bit(63))
    if not co[1] & pieces[5] & _bit(4):
        w = 0
    if not co[0] & pieces[5] & _bit(60):
        b = 0
    return w | b


def _parse_fen(fen: str):
    p = np.zeros((), K.POS_DTYPE)
    parts = fen.split()
    rows = parts[0].split("/")
    if len(rows) != 8:
        raise ValueError(f"invalid fen: {fen!r}")
    pieces, co = [0] * 6, [0, 0]
    for r, row in enumerate(rows):
        f = 0
        for ch in row:
            if ch.isdigit():
                f += int(ch)
            else:
                t = _SYMBOLS.find(ch.lower())
                if t < 0 or f > 7:
                    raise ValueError(f"invalid fen: {fen!r}")
                sq = (7 - r) * 8 + f
                pieces[t] |= _bit(sq)
                co[1 if ch.isupper() else 0] |= _bit(sq)
                f += 1
        if f != 8:
            raise ValueError(f"invalid fen: {fen!r}")
    p["pieces"] = pieces
    p["occupied_co"] = co
    p["turn"] = 1 if (len(parts) < 2 or parts[1] == "w") else 0
    cr = 0
    for ch in (parts[2] if len(parts) > 2 else "-"):
        cr |= {"K": _bit(7), "Q": _bit(0), "k": _bit(63), "q": _bit(56)}.get(ch, 0)
    p["castling_rights"] = cr
    p["castling_rights"] = _clean_castling(p)
    ep = parts[3] if len(parts) > 3 else "-"
    p["ep_square"] = -1 if ep == "-" else (int(ep[1]) - 1) * 8 + ord(ep[0]) - ord("a")
    p["halfmove_clock"] = int(parts[4]) if len(parts) > 4 else 0
    p["fullmove_number"] = int(parts[5]) if len(parts) > 5 else 1
    return p


def _piece_type_at(p, sq):
    for t in range(6):
        if int(p["pieces"][t]) >> sq & 1:
            return t + 1
    return 0


def _array(p):
    """board_fen_to_array (board.py:114-125): row 0 = rank 8, +type white, -type black."""
    a = np.zeros((8, 8), np.int8)
    white = int(p["occupied_co"][1])
    for r in range(8):
        for f in range(8):
            sq = (7 - r) * 8 + f
            t = _piece_type_at(p, sq)
            if t:
                a[r, f] = t if white >> sq & 1 else -t
    return a


class Board:
    def __init__(self, board_fen: Optional[str] = None, array: Optional[np.ndarray] = None,
                 history_size: int = 8):
        self.board_size = ConfigChess.board_size
        self.number_unique_pieces = ConfigChess.number_unique_pieces
        if array is not None:
            assert isinstance(array, np.ndarray)
            assert all(dim == self.board_size for dim in array.shape)
            assert np.unique(array).size <= self.number_unique_pieces + 1
            self.array = array.astype("int8")
            board_fen = self.array_to_board_fen(self.array)
        else:
            board_fen = ConfigChess.initial_board_fen if board_fen is None else board_fen
        self._pos = _parse_fen(self.get_fen(board_fen))
        if array is None:
            self.array = _array(self._pos)
        self._stack = []  # (transposition key, irreversible) per pushed move
        self.history_size = history_size
        self.state_history = _History(history_size)
        for _ in range(history_size):
            self.state_history.append(None)
        self.state_history.append(self._current_entry())

    # --------------------------------------------------------- reference API
    @property
    def array_one_hot(self) -> np.ndarray:
        return np.eye(self.number_unique_pieces + 1)[self.array]

    @property
    def moves(self) -> List[Move]:
        return [Move.from_code(c) for c in self._legal()[0]]

    @property
    def state(self) -> np.ndarray:
        return np.dstack([self.array_one_hot,
                          np.full((self.board_size, self.board_size), self.is_repetition())])

    @property
    def full_state(self) -> np.ndarray:
        """Board.full_state (board.py:55-73), encoded on the GPU; float64 like
        the reference (every value is a small integer)."""
        hist = np.zeros(K.HISTORY, K.POS_DTYPE)
        valid = np.zeros(K.HISTORY, np.uint8)
        entries = list(self.state_history.entries)
        for i, e in enumerate(entries[-K.HISTORY:]):
            if e is not None:
                hist[i], valid[i] = e, 1
        out = K.encode(hist[None], valid[None])[0].astype(np.float64)
        last = hist[K.HISTORY - 1].copy()
        last["repetition"] = 0
        if valid[-1] == 0 or not _same_position(last, self._pos):
            # the deque's last state is not this board (mirror()/copy() before
            # update_array): castling planes and counters come from the board
            hist[K.HISTORY - 1] = self._pos
            out[..., 112:] = K.encode(hist[None], valid[None])[0][..., 112:]
        return out

    @staticmethod
    def get_fen(board_fen: str):
        c = ConfigChess
        return " ".join([board_fen, c.initial_turn, c.initial_castling_rights, c.initial_ep_quare,
                         c.initial_halfmove_clock, c.initial_fullmove_number])

    @staticmethod
    def from_one_hot(array_oh: np.ndarray) -> np.ndarray:
        array = np.argmax(array_oh, axis=-1)
        big = np.where(array > ConfigChess.number_unique_pieces / 2)
        array[big] = array[big] - ConfigChess.number_unique_pieces + 1
        return array

    @staticmethod
    def piece_symbol_to_int(piece_symbol: Optional[str]) -> int:
        if piece_symbol is None:
            return 0
        piece_int = ConfigChess.piece_symbols.index(piece_symbol.lower())
        return (1 if piece_symbol.isupper() else -1) * piece_int

    @staticmethod
    def int_to_piece_symbol(piece_int: int) -> Optional[str]:
        player, sym = np.sign(piece_int), ConfigChess.piece_symbols[np.abs(piece_int)]
        if sym is None:
            return sym
        return sym if player < 0 else sym.upper()

    def legal_moves_mask(self, all_possible_moves: List[Move]) -> np.ndarray:
        """[move in self.moves for move in all_possible_moves] (board.py:111-112):
        the device mask when all_possible_moves is the action list."""
        codes, mask = self._legal()[:2]
        if len(all_possible_moves) == K.ACTIONS:
            from custom_alphazero.chess.utils import get_all_possible_moves
            if all_possible_moves == get_all_possible_moves():
                return mask
        legal = set(int(c) for c in codes)
        return np.asarray([m.code in legal for m in all_possible_moves])

    def board_fen_to_array(self, fen: str) -> np.ndarray:
        mat = []
        for elem in fen.replace("/", ""):
            if elem.isdigit():
                mat.extend(int(elem) * [0])
            else:
                mat.append(self.piece_symbol_to_int(elem))
        return np.asarray(mat).reshape((self.board_size, self.board_size)).astype("int8")

    def array_to_board_fen(self, array: np.ndarray) -> str:
        fen, cases, empty = "", 0, 0
        for piece_int in np.nditer(array):
            sym = self.int_to_piece_symbol(int(piece_int))
            if sym is None:
                empty += 1
            else:
                if empty > 0:
                    fen += str(empty)
                    empty = 0
                fen += sym
            cases += 1
            if cases % self.board_size == 0:
                if empty:
                    fen += str(empty)
                if cases != self.board_size * self.board_size:
                    fen += "/"
                empty = 0
        return fen

    def update_array(self):
        self.array = self.board_fen_to_array(self.board_fen())
        self.state_history.append(self._current_entry())

    def get_random_move(self) -> Optional[Move]:
        try:
            return np.random.choice(self.moves)
        except ValueError:
            return None

    def play(self, move: Move, on_copy: bool = False, keep_same_player: bool = False) -> "Board":
        board = self.copy() if on_copy else self
        board.push_uci(move.uci)
        if keep_same_player:
            board = board.mirror()
            board._pos["turn"] = 1  # virtually, it is always white to play
        board.update_array()
        if not on_copy:
            self.__dict__.update(board.__dict__)
        return board

    def play_random(self) -> "Board":
        return self.play(self.get_random_move())

    def get_result(self):
        if not self.is_game_over():
            return None
        result = self.result()
        if len(result) == 3:
            return 1 if result[0] > result[1] else -1
        elif len(result) == 7:
            return 0

    def display_ascii(self):
        for row in self.array:
            print("".join(map(lambda x: self.int_to_piece_symbol(x) if x else ".", row)))

    # ------------------------------------------------ python-chess subset
    @property
    def turn(self) -> bool:
        return bool(self._pos["turn"])

    @turn.setter
    def turn(self, value: bool):
        self._pos["turn"] = int(bool(value))

    @property
    def halfmove_clock(self) -> int:
        return int(self._pos["halfmove_clock"])

    @property
    def fullmove_number(self) -> int:
        return int(self._pos["fullmove_number"])

    @property
    def ep_square(self) -> Optional[int]:
        ep = int(self._pos["ep_square"])
        return None if ep < 0 else ep

    @property
    def castling_rights(self) -> int:
        return int(self._pos["castling_rights"])

    @property
    def legal_moves(self) -> List[Move]:
        return self.moves

    def clean_castling_rights(self) -> int:
        return _clean_castling(self._pos)

    def has_queenside_castling_rights(self, color: bool) -> bool:
        back = _RANK_1 if color else _RANK_8
        return bool(self.clean_castling_rights() & _FILE_A & back)

    def has_kingside_castling_rights(self, color: bool) -> bool:
        back = _RANK_1 if color else _RANK_8
        return bool(self.clean_castling_rights() & _FILE_H & back)

    def board_fen(self) -> str:
        return self.array_to_board_fen(_array(self._pos))

    def fen(self) -> str:
        cr = self.clean_castling_rights()
        castling = "".join(s for s, b in (("K", 7), ("Q", 0), ("k", 63), ("q", 56)) if cr >> b & 1)
        ep = self.ep_square if self.has_legal_en_passant() else None
        ep_s = "-" if ep is None else "abcdefgh"[ep & 7] + str((ep >> 3) + 1)
        return " ".join([self.board_fen(), "w" if self.turn else "b", castling or "-", ep_s,
                         str(self.halfmove_clock), str(self.fullmove_number)])

    def __repr__(self):
        return f"Board({self.fen()!r})"

    def __eq__(self, other):
        return isinstance(other, Board) and self._key() == other._key() and \
            self.halfmove_clock == other.halfmove_clock and \
            self.fullmove_number == other.fullmove_number

    def outcome_code(self) -> int:
        return int(self._legal()[2])

    def is_game_over(self) -> bool:
        return self.outcome_code() != 0

    def is_checkmate(self) -> bool:
        return self.outcome_code() == 1

    def is_insufficient_material(self) -> bool:
        return self.outcome_code() == 2

    def is_stalemate(self) -> bool:
        return self.outcome_code() == 3

    def result(self) -> str:
        code = self.outcome_code()
        if code == 0:
            return "*"
        if code == 1:
            return "0-1" if self.turn else "1-0"
        return "1/2-1/2"

    def has_legal_en_passant(self) -> bool:
        ep = int(self._pos["ep_square"])
        if ep < 0:
            return False
        pawns = int(self._pos["pieces"][0])
        for c in self._legal()[0]:
            f, t = int(c) & 63, (int(c) >> 6) & 63
            if t == ep and pawns >> f & 1 and abs(t - f) in (7, 9):
                return True
        return False

    def push_uci(self, uci: str):
        move = Move(uci=uci)
        codes = [int(c) for c in self._legal()[0]]
        if move.code not in codes:
            raise ValueError(f"illegal uci: {uci!r} in {self.fen()}")
        self.push(move)

    def push(self, move: Move):
        code = move.code
        f, t = code & 63, (code >> 6) & 63
        pieces = [int(x) for x in self._pos["pieces"]]
        touched = _bit(f) ^ _bit(t)
        opp = int(self._pos["occupied_co"][0 if self.turn else 1])
        zeroing = bool(touched & pieces[0] or touched & opp)
        cr = self.clean_castling_rights()
        kings_w = pieces[5] & int(self._pos["occupied_co"][1])
        kings_b = pieces[5] & int(self._pos["occupied_co"][0])
        reduces = bool(touched & cr or (cr & _RANK_1 and touched & kings_w)
                       or (cr & _RANK_8 and touched & kings_b))
        irreversible = zeroing or reduces or self.has_legal_en_passant()
        self._stack.append((self._key(), irreversible))
        self._pos = K.play(self._pos, code, keep_same_player=False)[0]
        self._legal_cache = None

    def is_repetition(self, count: int = 3) -> bool:
        """python-chess is_repetition: walk back through reversible moves."""
        key = self._key()
        i = len(self._stack)
        while True:
            if count <= 1:
                return True
            if i < count - 1:
                break
            i -= 1
            k, irreversible = self._stack[i]
            if irreversible:
                break
            if k == key:
                count -= 1
        return False

    def mirror(self) -> "Board":
        """python-chess mirror(): a copy (fresh __init__ state: start-position
        array and history), flipped vertically with colours and turn swapped,
        move stack cleared."""
        b = Board(history_size=self.history_size)
        p = self._pos.copy()
        p["pieces"] = [_bswap(x) for x in p["pieces"]]
        w, bl = _bswap(p["occupied_co"][1]), _bswap(p["occupied_co"][0])
        p["occupied_co"] = [w, bl]
        p["castling_rights"] = _bswap(p["castling_rights"])
        if int(p["ep_square"]) >= 0:
            p["ep_square"] = int(p["ep_square"]) ^ 56
        p["turn"] = 1 - int(p["turn"])
        p["repetition"] = 0
        b._pos = p
        return b

    def copy(self) -> "Board":
        """python-chess copy(): re-runs __init__ (start-position array and
        history, as the reference's subclass does), copies position and stack."""
        b = Board(history_size=self.history_size)
        b._pos = self._pos.copy()
        b._stack = list(self._stack)
        return b

    def __deepcopy__(self, memo):
        b = self.copy()
        memo[id(self)] = b
        return b

    # ------------------------------------------------------------- helpers
    def _legal(self):
        cache = getattr(self, "_legal_cache", None)
        if cache is not None and _same_position(cache[0], self._pos):
            return cache[1]
        moves, counts, mask, outcome = K.legal(self._pos)
        val = (moves[0, :counts[0]].copy(), mask[0], int(outcome[0]))
        self._legal_cache = (self._pos.copy(), val)
        return val

    def _key(self):
        """python-chess _transposition_key()."""
        p = self._pos
        ep = int(p["ep_square"]) if self.has_legal_en_passant() else -1
        return (tuple(int(x) for x in p["pieces"]), tuple(int(x) for x in p["occupied_co"]),
                int(p["turn"]), _clean_castling(p), ep)

    def _current_entry(self):
        e = self._pos.copy()
        e["repetition"] = int(self.is_repetition())
        return e


def _same_position(a, b):
    return bytes(np.asarray(a).tobytes()) == bytes(np.asarray(b).tobytes())


class _History:
    """state_history: the reference keeps a deque(maxlen=history_size) of
    state arrays; here the positions, encoded on demand (GPU).  Iterating
    yields the state arrays like the reference's deque."""

    def __init__(self, maxlen):
        self.entries = deque(maxlen=maxlen)

    def append(self, entry):
        self.entries.append(None if entry is None else np.asarray(entry).copy())

    def __len__(self):
        return len(self.entries)

    def __iter__(self):
        hist = np.zeros((len(self.entries), K.HISTORY), K.POS_DTYPE)
        valid = np.zeros((len(self.entries), K.HISTORY), np.uint8)
        for i, e in enumerate(self.entries):
            if e is not None:
                hist[i, -1], valid[i, -1] = e, 1
        states = K.encode(hist, valid)[:, :, :, 7 * 14:8 * 14].astype(np.float64) \
            if len(self.entries) else []
        return iter(list(states))
