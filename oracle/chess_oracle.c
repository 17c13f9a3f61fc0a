/*
 * chess_oracle.c -- CPU restatement of the reference's chess board path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/ (and __graft_entry__.smoke()) load
 * this library, as the checker of the HIP chess kernels (csrc/az_chess.hip);
 * it is never the product path.
 *
 * The reference (custom_alphazero/chess/board.py, move.py, utils.py) is a thin
 * subclass of python-chess 1.9.4 (poetry.lock:227-228), an un-vendored
 * dependency that is NOT installed here.  What is restated, from python-chess's
 * published algorithm (chess/__init__.py of that release):
 *   generate_legal_moves      legal move SET and generation ORDER: non-pawn
 *                             pieces by from-square descending (to-squares
 *                             descending), castling (h-side rook first),
 *                             pawn captures (Q,R,B,N promotions), single
 *                             pushes, double pushes, en passant; in check:
 *                             king evasions first, then captures/blocks, then
 *                             the en-passant capture of a checking pawn; the
 *                             _is_safe filter keeps the order.
 *   push                      counters, castling-right updates, ep square set
 *                             after every double push, ep capture, castling
 *                             as king-takes-rook internally, promotions.
 *   mirror                    flip_vertical + colour swap + turn flip; the
 *                             move stack is cleared (is_repetition() -> False)
 *   outcome                   checkmate, insufficient material, stalemate,
 *                             75-move rule, in that order (fivefold repetition
 *                             never fires: mirror clears the stack).
 * and from the reference itself:
 *   Board.play(keep_same_player=True)   chess/board.py:162-173 (push, mirror,
 *                             turn = True)
 *   Board.array                board_fen_to_array, chess/board.py:114-125
 *   Board.state / full_state   chess/board.py:43-73 (eye(13)[array] + the
 *                             repetition plane per history entry, then four
 *                             castling planes, fullmove, halfmove)
 *   legal_moves_mask          chess/board.py:111-112 over
 *   get_all_possible_moves    chess/utils.py:11-32 (queen + knight moves from
 *                             every square, white promotions; sorted by
 *                             Move.__lt__ = (pos_from, pos_to) tuples,
 *                             chess/move.py:33-37)
 *
 * Parity pin: the legal move SET (and push) is pinned by published perft
 * node counts (tests/test_chess_oracle.py: start position, "Kiwipete" and
 * the other standard perft positions).  The generation ORDER, the history
 * planes and the outcome rules follow python-chess's published algorithm but
 * are "parity unpinned": python-chess is absent here and the reference holds
 * no chess fixture.
 *
 * Squares follow python-chess: A1 = 0 .. H8 = 63, file = sq & 7, rank = sq >> 3.
 * Moves are uint16: from | to << 6 | promotion << 12 (python-chess piece type,
 * 0 = none, 2..5 = N,B,R,Q).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t bb_t;

/* identical layout to az_chess_pos (include/az_chess.h) */
typedef struct {
    bb_t pieces[6];       /* pawns, knights, bishops, rooks, queens, kings */
    bb_t occupied_co[2];  /* [0] BLACK, [1] WHITE */
    bb_t castling_rights; /* rook squares */
    int16_t ep_square;    /* -1 = None */
    uint8_t turn;         /* 1 = WHITE */
    uint8_t repetition;
    uint16_t halfmove_clock;
    uint16_t fullmove_number;
} cpos;

enum { PAWN = 1, KNIGHT, BISHOP, ROOK, QUEEN, KING };
#define BBS(s) (1ULL << (s))
#define RANK_1 0xFFULL
#define RANK_8 0xFF00000000000000ULL
#define FILE_A 0x0101010101010101ULL
#define FILE_H 0x8080808080808080ULL
#define DARK 0xAA55AA55AA55AA55ULL

static int msb(bb_t x) { return 63 - __builtin_clzll(x); }
static int popcnt(bb_t x) { return __builtin_popcountll(x); }
static bb_t occupied(const cpos* p) { return p->occupied_co[0] | p->occupied_co[1]; }

static bb_t KNIGHT_ATT[64], KING_ATT[64], PAWN_ATT[2][64];
static bb_t RAYS[64][64], BETWEEN[64][64];
static int g_init = 0;

static bb_t step_set(int sq, const int (*d)[2], int nd) {
    bb_t r = 0;
    int f = sq & 7, k = sq >> 3;
    for (int i = 0; i < nd; ++i) {
        int ff = f + d[i][0], kk = k + d[i][1];
        if (ff >= 0 && ff < 8 && kk >= 0 && kk < 8) r |= BBS(kk * 8 + ff);
    }
    return r;
}

static void init_tables(void) {
    if (g_init) return;
    static const int kn[8][2] = {{1, 2}, {2, 1}, {2, -1}, {1, -2}, {-1, -2}, {-2, -1}, {-2, 1}, {-1, 2}};
    static const int kg[8][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
    static const int pw[2][2] = {{-1, 1}, {1, 1}};
    static const int pb[2][2] = {{-1, -1}, {1, -1}};
    for (int s = 0; s < 64; ++s) {
        KNIGHT_ATT[s] = step_set(s, kn, 8);
        KING_ATT[s] = step_set(s, kg, 8);
        PAWN_ATT[1][s] = step_set(s, pw, 2);
        PAWN_ATT[0][s] = step_set(s, pb, 2);
    }
    /* RAYS[a][b]: the whole line through a and b (python-chess BB_RAYS);
     * BETWEEN[a][b]: squares strictly between them (python-chess between()) */
    for (int a = 0; a < 64; ++a)
        for (int b = 0; b < 64; ++b) {
            RAYS[a][b] = BETWEEN[a][b] = 0;
            if (a == b) continue;
            int df = (b & 7) - (a & 7), dk = (b >> 3) - (a >> 3);
            int sf = (df > 0) - (df < 0), sk = (dk > 0) - (dk < 0);
            if (!(df == 0 || dk == 0 || df == dk || df == -dk)) continue;
            bb_t line = BBS(a);
            for (int dir = -1; dir <= 1; dir += 2) {
                int f = (a & 7) + dir * sf, k = (a >> 3) + dir * sk;
                while (f >= 0 && f < 8 && k >= 0 && k < 8) {
                    line |= BBS(k * 8 + f);
                    f += dir * sf;
                    k += dir * sk;
                }
            }
            RAYS[a][b] = line;
            int f = (a & 7) + sf, k = (a >> 3) + sk;
            while (k * 8 + f != b) {
                BETWEEN[a][b] |= BBS(k * 8 + f);
                f += sf;
                k += sk;
            }
        }
    g_init = 1;
}

static bb_t slide(int sq, bb_t occ, int diag) {
    static const int rd[4][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}};
    static const int bd[4][2] = {{1, 1}, {1, -1}, {-1, 1}, {-1, -1}};
    const int(*d)[2] = diag ? bd : rd;
    bb_t r = 0;
    for (int i = 0; i < 4; ++i) {
        int f = (sq & 7) + d[i][0], k = (sq >> 3) + d[i][1];
        while (f >= 0 && f < 8 && k >= 0 && k < 8) {
            int s = k * 8 + f;
            r |= BBS(s);
            if (occ & BBS(s)) break;
            f += d[i][0];
            k += d[i][1];
        }
    }
    return r;
}

static int piece_type_at(const cpos* p, int sq) {
    for (int t = 0; t < 6; ++t)
        if (p->pieces[t] & BBS(sq)) return t + 1;
    return 0;
}

/* python-chess attacks_mask(square) */
static bb_t attacks_mask(const cpos* p, int sq) {
    bb_t s = BBS(sq), occ = occupied(p);
    if (s & p->pieces[PAWN - 1]) return PAWN_ATT[(p->occupied_co[1] & s) ? 1 : 0][sq];
    if (s & p->pieces[KNIGHT - 1]) return KNIGHT_ATT[sq];
    if (s & p->pieces[KING - 1]) return KING_ATT[sq];
    bb_t a = 0;
    if (s & (p->pieces[BISHOP - 1] | p->pieces[QUEEN - 1])) a |= slide(sq, occ, 1);
    if (s & (p->pieces[ROOK - 1] | p->pieces[QUEEN - 1])) a |= slide(sq, occ, 0);
    return a;
}

/* python-chess _attackers_mask(color, square, occupied) */
static bb_t attackers(const cpos* p, int color, int sq, bb_t occ) {
    bb_t qr = p->pieces[QUEEN - 1] | p->pieces[ROOK - 1];
    bb_t qb = p->pieces[QUEEN - 1] | p->pieces[BISHOP - 1];
    bb_t a = (KING_ATT[sq] & p->pieces[KING - 1]) | (KNIGHT_ATT[sq] & p->pieces[KNIGHT - 1]) |
             (slide(sq, occ, 0) & qr) | (slide(sq, occ, 1) & qb) |
             (PAWN_ATT[!color][sq] & p->pieces[PAWN - 1]);
    return a & p->occupied_co[color];
}

static int king_sq(const cpos* p, int color) {
    bb_t k = p->pieces[KING - 1] & p->occupied_co[color];
    return k ? msb(k) : -1;
}

/* python-chess clean_castling_rights() (standard chess) */
static bb_t clean_castling(const cpos* p) {
    bb_t c = p->castling_rights & p->pieces[ROOK - 1];
    bb_t w = c & RANK_1 & p->occupied_co[1] & (BBS(0) | BBS(7));
    bb_t b = c & RANK_8 & p->occupied_co[0] & (BBS(56) | BBS(63));
    if (!(p->occupied_co[1] & p->pieces[KING - 1] & BBS(4))) w = 0;
    if (!(p->occupied_co[0] & p->pieces[KING - 1] & BBS(60))) b = 0;
    return w | b;
}

typedef struct {
    uint16_t* m;
    int n;
} mlist;

static void add(mlist* L, int from, int to, int promo) {
    L->m[L->n++] = (uint16_t)(from | (to << 6) | (promo << 12));
}

static void add_pawn(mlist* L, int from, int to) {
    int r = to >> 3;
    if (r == 0 || r == 7) {
        add(L, from, to, QUEEN);
        add(L, from, to, ROOK);
        add(L, from, to, BISHOP);
        add(L, from, to, KNIGHT);
    } else {
        add(L, from, to, 0);
    }
}

static int attacked_for_king(const cpos* p, bb_t path, bb_t occ) {
    for (bb_t x = path; x; x &= ~BBS(msb(x)))
        if (attackers(p, !p->turn, msb(x), occ)) return 1;
    return 0;
}

/* python-chess generate_castling_moves */
static void gen_castling(const cpos* p, bb_t from_mask, bb_t to_mask, mlist* L) {
    int t = p->turn;
    bb_t back = t ? RANK_1 : RANK_8;
    bb_t king = p->occupied_co[t] & p->pieces[KING - 1] & back & from_mask;
    king &= (~king + 1);
    if (!king) return;
    int ks = msb(king);
    bb_t occ = occupied(p);
    int cfile = t ? 2 : 58, dfile = t ? 3 : 59, ffile = t ? 5 : 61, gfile = t ? 6 : 62;
    for (bb_t cand = clean_castling(p) & back & to_mask; cand; cand &= ~BBS(msb(cand))) {
        int rs = msb(cand);
        bb_t rook = BBS(rs);
        int a_side = rook < king;
        int kto = a_side ? cfile : gfile, rto = a_side ? dfile : ffile;
        bb_t king_path = BETWEEN[ks][kto], rook_path = BETWEEN[rs][rto];
        if (!(((occ ^ king ^ rook) & (king_path | rook_path | BBS(kto) | BBS(rto))) ||
              attacked_for_king(p, king_path | king, occ ^ king) ||
              attacked_for_king(p, BBS(kto), occ ^ king ^ rook ^ BBS(rto))))
            add(L, ks, kto, 0); /* _from_chess960: e1h1 -> e1g1 */
    }
}

static void gen_ep(const cpos* p, bb_t from_mask, bb_t to_mask, mlist* L) {
    int ep = p->ep_square;
    if (ep < 0 || !(BBS(ep) & to_mask)) return;
    if (BBS(ep) & occupied(p)) return;
    int t = p->turn;
    bb_t cap = p->pieces[PAWN - 1] & p->occupied_co[t] & from_mask & PAWN_ATT[!t][ep] &
               (0xFFULL << (8 * (t ? 4 : 3)));
    for (; cap; cap &= ~BBS(msb(cap))) add(L, msb(cap), ep, 0);
}

/* python-chess generate_pseudo_legal_moves */
static void gen_pseudo(const cpos* p, bb_t from_mask, bb_t to_mask, mlist* L) {
    int t = p->turn;
    bb_t own = p->occupied_co[t], occ = occupied(p);
    bb_t pawns_all = p->pieces[PAWN - 1];
    for (bb_t np = own & ~pawns_all & from_mask; np; np &= ~BBS(msb(np))) {
        int f = msb(np);
        for (bb_t mv = attacks_mask(p, f) & ~own & to_mask; mv; mv &= ~BBS(msb(mv))) add(L, f, msb(mv), 0);
    }
    if (from_mask & p->pieces[KING - 1]) gen_castling(p, from_mask, to_mask, L);
    bb_t pawns = pawns_all & own & from_mask;
    if (!pawns) return;
    for (bb_t c = pawns; c; c &= ~BBS(msb(c))) {
        int f = msb(c);
        for (bb_t tg = PAWN_ATT[t][f] & p->occupied_co[!t] & to_mask; tg; tg &= ~BBS(msb(tg)))
            add_pawn(L, f, msb(tg));
    }
    bb_t single, dbl;
    if (t) {
        single = (pawns << 8) & ~occ;
        dbl = (single << 8) & ~occ & (0xFFULL << 16 | 0xFFULL << 24);
    } else {
        single = (pawns >> 8) & ~occ;
        dbl = (single >> 8) & ~occ & (0xFFULL << 40 | 0xFFULL << 32);
    }
    single &= to_mask;
    dbl &= to_mask;
    for (; single; single &= ~BBS(msb(single))) {
        int to = msb(single);
        add_pawn(L, to + (t ? -8 : 8), to);
    }
    for (; dbl; dbl &= ~BBS(msb(dbl))) {
        int to = msb(dbl);
        add(L, to + (t ? -16 : 16), to, 0);
    }
    if (p->ep_square >= 0) gen_ep(p, from_mask, to_mask, L);
}

/* python-chess _generate_evasions */
static void gen_evasions(const cpos* p, int king, bb_t checkers, mlist* L) {
    int t = p->turn;
    bb_t sliders = checkers & (p->pieces[BISHOP - 1] | p->pieces[ROOK - 1] | p->pieces[QUEEN - 1]);
    bb_t attacked = 0;
    for (bb_t s = sliders; s; s &= ~BBS(msb(s))) attacked |= RAYS[king][msb(s)] & ~BBS(msb(s));
    for (bb_t mv = KING_ATT[king] & ~p->occupied_co[t] & ~attacked; mv; mv &= ~BBS(msb(mv)))
        add(L, king, msb(mv), 0);
    int checker = msb(checkers);
    if (BBS(checker) == checkers) {
        bb_t target = BETWEEN[king][checker] | checkers;
        gen_pseudo(p, ~p->pieces[KING - 1], target, L);
        if (p->ep_square >= 0 && !(BBS(p->ep_square) & target)) {
            int last_double = p->ep_square + (t ? -8 : 8);
            if (last_double == checker) gen_ep(p, ~0ULL, ~0ULL, L);
        }
    }
}

static bb_t slider_blockers(const cpos* p, int king) {
    bb_t rq = p->pieces[ROOK - 1] | p->pieces[QUEEN - 1];
    bb_t bq = p->pieces[BISHOP - 1] | p->pieces[QUEEN - 1];
    bb_t snipers = (slide(king, 0, 0) & rq) | (slide(king, 0, 1) & bq);
    bb_t blockers = 0, occ = occupied(p);
    for (bb_t s = snipers & p->occupied_co[!p->turn]; s; s &= ~BBS(msb(s))) {
        bb_t b = BETWEEN[king][msb(s)] & occ;
        if (b && BBS(msb(b)) == b) blockers |= b;
    }
    return blockers & p->occupied_co[p->turn];
}

/* python-chess pin_mask(color, square) */
static bb_t pin_mask(const cpos* p, int color, int sq) {
    int king = king_sq(p, color);
    if (king < 0) return ~0ULL;
    bb_t sm = BBS(sq), occ = occupied(p);
    bb_t rq = p->pieces[ROOK - 1] | p->pieces[QUEEN - 1], bq = p->pieces[BISHOP - 1] | p->pieces[QUEEN - 1];
    bb_t file = FILE_A << (king & 7), rank = RANK_1 << (8 * (king >> 3));
    bb_t rays[3] = {slide(king, 0, 0) & file, slide(king, 0, 0) & rank, slide(king, 0, 1)};
    bb_t sl[3] = {rq, rq, bq};
    for (int i = 0; i < 3; ++i) {
        if (rays[i] & sm) {
            for (bb_t sn = rays[i] & sl[i] & p->occupied_co[!color]; sn; sn &= ~BBS(msb(sn))) {
                int s = msb(sn);
                if ((BETWEEN[s][king] & (occ | sm)) == sm) return RAYS[king][s];
            }
            break;
        }
    }
    return ~0ULL;
}

static int ep_skewered(const cpos* p, int king, int capturer) {
    int t = p->turn;
    int last_double = p->ep_square + (t ? -8 : 8);
    bb_t occ = (occupied(p) & ~BBS(last_double) & ~BBS(capturer)) | BBS(p->ep_square);
    bb_t rank = RANK_1 << (8 * (king >> 3));
    bb_t horiz = p->occupied_co[!t] & (p->pieces[ROOK - 1] | p->pieces[QUEEN - 1]);
    if (slide(king, occ, 0) & rank & horiz) return 1;
    bb_t diag = p->occupied_co[!t] & (p->pieces[BISHOP - 1] | p->pieces[QUEEN - 1]);
    if (slide(king, occ, 1) & diag) return 1;
    return 0;
}

static int is_safe(const cpos* p, int king, bb_t blockers, uint16_t m) {
    int from = m & 63, to = (m >> 6) & 63;
    if (from == king) {
        /* is_castling: the king moves more than one file */
        int diff = (from & 7) - (to & 7);
        if (diff > 1 || diff < -1) return 1;
        return !attackers(p, !p->turn, to, occupied(p));
    }
    int is_ep = p->ep_square == to && (p->pieces[PAWN - 1] & BBS(from)) &&
                (abs(to - from) == 7 || abs(to - from) == 9) && !(occupied(p) & BBS(to));
    if (is_ep) return (pin_mask(p, p->turn, from) & BBS(to)) && !ep_skewered(p, king, from);
    return !(blockers & BBS(from)) || (RAYS[from][to] & BBS(king));
}

/* python-chess generate_legal_moves -> count; moves in generation order */
int orc_chess_legal(const cpos* p, uint16_t* out) {
    init_tables();
    uint16_t buf[512];
    mlist L = {buf, 0};
    int king = king_sq(p, p->turn);
    if (king < 0) {
        L.m = out;
        gen_pseudo(p, ~0ULL, ~0ULL, &L);
        return L.n;
    }
    bb_t blockers = slider_blockers(p, king);
    bb_t checkers = attackers(p, !p->turn, king, occupied(p));
    if (checkers)
        gen_evasions(p, king, checkers, &L);
    else
        gen_pseudo(p, ~0ULL, ~0ULL, &L);
    int n = 0;
    for (int i = 0; i < L.n; ++i)
        if (is_safe(p, king, blockers, buf[i])) out[n++] = buf[i];
    return n;
}

static void remove_piece(cpos* p, int sq) {
    for (int t = 0; t < 6; ++t) p->pieces[t] &= ~BBS(sq);
    p->occupied_co[0] &= ~BBS(sq);
    p->occupied_co[1] &= ~BBS(sq);
}

static void set_piece(cpos* p, int sq, int type, int color) {
    remove_piece(p, sq);
    p->pieces[type - 1] |= BBS(sq);
    p->occupied_co[color] |= BBS(sq);
}

/* python-chess Board.push (standard chess; the move is legal) */
void orc_chess_push(cpos* p, uint16_t m) {
    init_tables();
    int from = m & 63, to = (m >> 6) & 63, promo = m >> 12;
    int t = p->turn;
    /* _to_chess960: standard castling e1g1 / e1c1 -> king takes rook */
    int e = t ? 4 : 60;
    if (from == e && (p->pieces[KING - 1] & BBS(e))) {
        if (to == e + 2 && !(p->pieces[ROOK - 1] & BBS(e + 2))) to = e + 3;
        else if (to == e - 2 && !(p->pieces[ROOK - 1] & BBS(e - 2))) to = e - 4;
    }
    p->castling_rights = clean_castling(p);
    int ep = p->ep_square;
    p->ep_square = -1;
    p->halfmove_clock++;
    if (!t) p->fullmove_number++;
    bb_t touched = BBS(from) ^ BBS(to);
    if ((touched & p->pieces[PAWN - 1]) || (touched & p->occupied_co[!t])) p->halfmove_clock = 0;
    bb_t from_bb = BBS(from), to_bb = BBS(to);
    int piece = piece_type_at(p, from);
    remove_piece(p, from);
    int captured = piece_type_at(p, to);
    p->castling_rights &= ~to_bb & ~from_bb;
    if (piece == KING) p->castling_rights &= ~(t ? RANK_1 : RANK_8);
    if (piece == PAWN) {
        int diff = to - from;
        if (diff == 16 && (from >> 3) == 1) p->ep_square = (int16_t)(from + 8);
        else if (diff == -16 && (from >> 3) == 6) p->ep_square = (int16_t)(from - 8);
        else if (to == ep && (diff == 7 || diff == 9 || diff == -7 || diff == -9) && !captured)
            remove_piece(p, ep + (t ? -8 : 8));
    }
    if (promo) piece = promo;
    int castling = piece == KING && (p->occupied_co[t] & to_bb);
    if (castling) {
        int a_side = (to & 7) < (from & 7);
        remove_piece(p, from);
        remove_piece(p, to);
        int base = t ? 0 : 56;
        if (a_side) {
            set_piece(p, base + 2, KING, t);
            set_piece(p, base + 3, ROOK, t);
        } else {
            set_piece(p, base + 6, KING, t);
            set_piece(p, base + 5, ROOK, t);
        }
    } else {
        set_piece(p, to, piece, t);
    }
    p->turn = (uint8_t)!t;
    p->repetition = 0;
}

static bb_t flip_vertical(bb_t x) { return __builtin_bswap64(x); }

/* python-chess Board.mirror(): flip_vertical, swap colours, flip turn; the
 * stack is cleared so is_repetition() is False */
void orc_chess_mirror(cpos* p) {
    for (int t = 0; t < 6; ++t) p->pieces[t] = flip_vertical(p->pieces[t]);
    bb_t w = flip_vertical(p->occupied_co[1]), b = flip_vertical(p->occupied_co[0]);
    p->occupied_co[1] = b;
    p->occupied_co[0] = w;
    p->castling_rights = flip_vertical(p->castling_rights);
    if (p->ep_square >= 0) p->ep_square = (int16_t)(p->ep_square ^ 56);
    p->turn = (uint8_t)!p->turn;
    p->repetition = 0;
}

/* Board.play(move, keep_same_player=True) (chess/board.py:162-173) */
void orc_chess_play_canonical(cpos* p, uint16_t m) {
    orc_chess_push(p, m);
    orc_chess_mirror(p);
    p->turn = 1;
}

static int insufficient_color(const cpos* p, int c) {
    bb_t own = p->occupied_co[c], opp = p->occupied_co[!c];
    if (own & (p->pieces[PAWN - 1] | p->pieces[ROOK - 1] | p->pieces[QUEEN - 1])) return 0;
    if (own & p->pieces[KNIGHT - 1])
        return popcnt(own) <= 2 && !(opp & ~p->pieces[KING - 1] & ~p->pieces[QUEEN - 1]);
    if (own & p->pieces[BISHOP - 1]) {
        bb_t bi = p->pieces[BISHOP - 1];
        int same = !(bi & DARK) || !(bi & ~DARK);
        return same && !p->pieces[PAWN - 1] && !p->pieces[KNIGHT - 1];
    }
    return 1;
}

/* python-chess outcome() termination: 0 none, 1 checkmate, 2 insufficient
 * material, 3 stalemate, 4 seventy-five moves */
int orc_chess_outcome(const cpos* p) {
    uint16_t buf[256];
    int n = orc_chess_legal(p, buf);
    int king = king_sq(p, p->turn);
    int check = king >= 0 && attackers(p, !p->turn, king, occupied(p));
    if (check && n == 0) return 1;
    if (insufficient_color(p, 0) && insufficient_color(p, 1)) return 2;
    if (n == 0) return 3;
    if (p->halfmove_clock >= 150) return 4;
    return 0;
}

uint64_t orc_chess_perft(const cpos* p, int depth) {
    uint16_t buf[256];
    int n = orc_chess_legal(p, buf);
    if (depth <= 1) return depth == 1 ? (uint64_t)n : 1;
    uint64_t s = 0;
    for (int i = 0; i < n; ++i) {
        cpos q = *p;
        orc_chess_push(&q, buf[i]);
        s += orc_chess_perft(&q, depth - 1);
    }
    return s;
}

/* Board.array (board_fen_to_array, chess/board.py:114-125): row 0 = rank 8,
 * +piece type for white, -piece type for black */
void orc_chess_array(const cpos* p, int8_t* out) {
    for (int r = 0; r < 8; ++r)
        for (int f = 0; f < 8; ++f) {
            int sq = (7 - r) * 8 + f;
            int t = piece_type_at(p, sq);
            out[r * 8 + f] = (int8_t)(t == 0 ? 0 : ((p->occupied_co[1] & BBS(sq)) ? t : -t));
        }
}

/* Board.full_state (chess/board.py:55-73) from an explicit history:
 * hist[0..7] oldest first (the deque), valid[h] = 0 for the zero-filled
 * entries; castling planes and counters come from `cur` (the board itself).
 * out: [8][8][118] float64. */
void orc_chess_full_state(const cpos* hist, const uint8_t* valid, const cpos* cur, double* out) {
    memset(out, 0, sizeof(double) * 64 * 118);
    for (int h = 0; h < 8; ++h) {
        if (!valid[h]) continue;
        int8_t a[64];
        orc_chess_array(&hist[h], a);
        for (int i = 0; i < 64; ++i) {
            int idx = a[i] >= 0 ? a[i] : 13 + a[i]; /* np.eye(13)[array] */
            out[i * 118 + h * 14 + idx] = 1.0;
            out[i * 118 + h * 14 + 13] = hist[h].repetition;
        }
    }
    bb_t c = clean_castling(cur);
    int t = cur->turn;
    bb_t back_t = t ? RANK_1 : RANK_8, back_o = t ? RANK_8 : RANK_1;
    double feat[6] = {(c & FILE_A & back_t) != 0, (c & FILE_H & back_t) != 0,
                      (c & FILE_A & back_o) != 0, (c & FILE_H & back_o) != 0,
                      cur->fullmove_number, cur->halfmove_clock};
    for (int i = 0; i < 64; ++i)
        for (int k = 0; k < 6; ++k) out[i * 118 + 112 + k] = feat[k];
}

/* ---- get_all_possible_moves (chess/utils.py:11-32) ---- */
static int promo_rank(int promo) {
    /* Move.__lt__ compares the promotion strings: "" < "b" < "n" < "q" < "r" */
    switch (promo) {
        case 0: return 0;
        case BISHOP: return 1;
        case KNIGHT: return 2;
        case QUEEN: return 3;
        default: return 4; /* ROOK */
    }
}

static int move_key(uint16_t m) {
    int from = m & 63, to = (m >> 6) & 63, promo = m >> 12;
    /* pos_from = (file, rank), pos_to = (file, rank, promo) */
    return ((((from & 7) * 8 + (from >> 3)) * 8 + (to & 7)) * 8 + (to >> 3)) * 5 + promo_rank(promo);
}

static int cmp_moves(const void* a, const void* b) {
    return move_key(*(const uint16_t*)a) - move_key(*(const uint16_t*)b);
}

static void empty_pos(cpos* p) {
    memset(p, 0, sizeof(*p));
    p->ep_square = -1;
    p->turn = 1;
    p->fullmove_number = 1;
}

static int add_unique(uint16_t* all, int n, const uint16_t* mv, int k) {
    for (int i = 0; i < k; ++i) {
        int seen = 0;
        for (int j = 0; j < n && !seen; ++j) seen = all[j] == mv[i];
        if (!seen) all[n++] = mv[i];
    }
    return n;
}

int orc_chess_all_moves(uint16_t* out) {
    init_tables();
    static uint16_t all[4096];
    uint16_t mv[512];
    int n = 0;
    cpos p;
    for (int sq = 0; sq < 64; ++sq)
        for (int piece = 0; piece < 2; ++piece) {
            empty_pos(&p);
            set_piece(&p, sq, piece ? KNIGHT : QUEEN, 1);
            n = add_unique(all, n, mv, orc_chess_legal(&p, mv));
        }
    /* underpromotions: white pawns on rank 7 (array row 1), then black pawns
     * on rank 8 (array row 0) to capture */
    empty_pos(&p);
    for (int f = 0; f < 8; ++f) set_piece(&p, 48 + f, PAWN, 1);
    n = add_unique(all, n, mv, orc_chess_legal(&p, mv));
    for (int f = 0; f < 8; ++f) set_piece(&p, 56 + f, PAWN, 0);
    n = add_unique(all, n, mv, orc_chess_legal(&p, mv));
    qsort(all, (size_t)n, sizeof(uint16_t), cmp_moves);
    memcpy(out, all, sizeof(uint16_t) * (size_t)n);
    return n;
}

/* Board.legal_moves_mask(all_possible_moves) (chess/board.py:111-112) */
void orc_chess_legal_mask(const cpos* p, const uint16_t* all, int n_all, uint8_t* mask) {
    uint16_t mv[256];
    int n = orc_chess_legal(p, mv);
    for (int i = 0; i < n_all; ++i) {
        mask[i] = 0;
        for (int j = 0; j < n; ++j)
            if (mv[j] == all[i]) mask[i] = 1;
    }
}

/* FEN -> position (python-chess set_fen for standard chess) */
int orc_chess_from_fen(const char* fen, cpos* p) {
    init_tables();
    memset(p, 0, sizeof(*p));
    p->ep_square = -1;
    p->turn = 1;
    p->fullmove_number = 1;
    int r = 7, f = 0;
    const char* c = fen;
    for (; *c && *c != ' '; ++c) {
        if (*c == '/') {
            r--;
            f = 0;
        } else if (*c >= '1' && *c <= '8') {
            f += *c - '0';
        } else {
            const char* sym = "pnbrqk";
            const char* q = NULL;
            for (int i = 0; i < 6; ++i)
                if ((*c | 32) == sym[i]) q = sym + i;
            if (!q || r < 0 || f > 7) return -1;
            set_piece(p, r * 8 + f, (int)(q - sym) + 1, (*c & 32) ? 0 : 1);
            f++;
        }
    }
    if (*c == ' ') c++;
    if (*c) {
        p->turn = *c == 'w';
        c++;
    }
    if (*c == ' ') c++;
    for (; *c && *c != ' '; ++c) {
        if (*c == 'K') p->castling_rights |= BBS(7);
        if (*c == 'Q') p->castling_rights |= BBS(0);
        if (*c == 'k') p->castling_rights |= BBS(63);
        if (*c == 'q') p->castling_rights |= BBS(56);
    }
    p->castling_rights = clean_castling(p);
    if (*c == ' ') c++;
    if (*c && *c != '-') {
        p->ep_square = (int16_t)((c[1] - '1') * 8 + (c[0] - 'a'));
        c += 2;
    } else if (*c) {
        c++;
    }
    if (*c == ' ') c++;
    if (*c) p->halfmove_clock = (uint16_t)strtol(c, (char**)&c, 10);
    if (*c == ' ') c++;
    if (*c) p->fullmove_number = (uint16_t)strtol(c, (char**)&c, 10);
    return 0;
}

int orc_chess_pos_size(void) { return (int)sizeof(cpos); }

/* =====================================================================
 * Chess self-play MCTS (BASELINE configs[4]), restating
 *   MCTS.select / search / evaluate_and_expand / backup / play
 *                                custom_alphazero/mcts/mcts.py:111-222
 *   normalize_probabilities     custom_alphazero/mcts/utils.py:4-16
 *   play_game                   custom_alphazero/self_play.py:37-82
 * over the chess rules above.  The tree arithmetic is the Connect-N
 * oracle's (az_oracle.c, linked in): float64 UCB with libm pow, first-max
 * argmax, float32 pairwise prior normalisation, positional zip of the
 * action-ordered priors with the python-chess move order (mcts.py:151),
 * float64 backup, np.random.choice on MT19937.  The reference cannot finish
 * a chess game under MCTS (chess Board.get_result() takes no
 * keep_same_player, chess/board.py:178 vs mcts.py:179): terminal boards
 * score as get_result does in the canonical form (checkmate 1, draw 0).
 * Games stop after max_plies (termination 5), a cap the reference lacks.
 * ===================================================================== */
#include <math.h>

typedef struct {
    uint32_t mt[624];
    int pos;
} orc_mt; /* az_oracle.c */
void orc_mt_seed(orc_mt* s, uint32_t seed);
double orc_mt_uniform(orc_mt* s);
int orc_normalize_f32(const float* p, int n, double* out);
void orc_normalize_f64(const double* p, int n, double* out);
double orc_pow_half(int64_t n);

#define ORC_CHESS_ACTIONS 1880

typedef struct {
    double W, prior;
    int64_t N;
    int child;       /* node id */
    uint16_t action; /* move code */
} cedge;

typedef struct {
    int first, count; /* edges (count 0: unexpanded or terminal) */
    int initial;      /* the game's Board(): history [0 x 7, state] */
    cpos pos;
} cnode;

typedef struct {
    cnode* nodes;
    cedge* edges;
    int n_nodes, cap_nodes, n_edges, cap_edges;
    double c_puct;
    int eval_kind; /* 0 synthetic, 1 callback */
    int (*cb)(void* ctx, const cpos* pos, int initial, float* probs, float* value);
    void* ctx;
    int64_t expansions, terminal_visits;
    int error;
} ctree;

static uint64_t c_splitmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* synthetic evaluator: dyadic priors k/64, values k/128, from a hash of
 * what the network would see (position, counters, root-history flag) */
void orc_chess_synth(const cpos* p, int initial, float* probs, float* value) {
    uint64_t h = c_splitmix(p->pieces[0]);
    for (int i = 1; i < 6; ++i) h = c_splitmix(h ^ p->pieces[i]);
    h = c_splitmix(h ^ p->occupied_co[0]);
    h = c_splitmix(h ^ p->occupied_co[1]);
    h = c_splitmix(h ^ p->castling_rights);
    uint64_t misc = (uint64_t)(uint16_t)p->ep_square | ((uint64_t)p->halfmove_clock << 16) |
                    ((uint64_t)p->fullmove_number << 32) | ((uint64_t)initial << 48);
    h = c_splitmix(h ^ misc);
    uint64_t vh = c_splitmix(h ^ 0x5555555555555555ull);
    *value = (float)(((double)(vh >> 56) - 128.0) / 128.0);
    if ((vh & 0x3F) == 0) {
        for (int a = 0; a < ORC_CHESS_ACTIONS; ++a) probs[a] = 0.0f;
        return;
    }
    uint64_t w = h;
    for (int a = 0; a < ORC_CHESS_ACTIONS; ++a) {
        if (a && a % 12 == 0) w = c_splitmix(w);
        probs[a] = (float)((double)(((w >> (5 * (a % 12))) & 31) + 1) / 64.0);
    }
}

static int g_lut_ready = 0;
static int16_t g_lut[64 * 64 * 5];
static int action_index(uint16_t m) {
    if (!g_lut_ready) {
        uint16_t all[2048];
        int n = orc_chess_all_moves(all);
        for (int i = 0; i < 64 * 64 * 5; ++i) g_lut[i] = -1;
        for (int i = 0; i < n; ++i) {
            int pr = all[i] >> 12;
            g_lut[((all[i] & 63) * 64 + ((all[i] >> 6) & 63)) * 5 + (pr ? pr - 1 : 0)] = (int16_t)i;
        }
        g_lut_ready = 1;
    }
    int pr = m >> 12;
    return g_lut[((m & 63) * 64 + ((m >> 6) & 63)) * 5 + (pr ? pr - 1 : 0)];
}

static int ct_new_node(ctree* t, const cpos* pos, int initial) {
    if (t->n_nodes == t->cap_nodes) {
        t->cap_nodes = t->cap_nodes ? 2 * t->cap_nodes : 4096;
        t->nodes = (cnode*)realloc(t->nodes, sizeof(cnode) * (size_t)t->cap_nodes);
    }
    int id = t->n_nodes++;
    t->nodes[id].first = 0;
    t->nodes[id].count = 0;
    t->nodes[id].initial = initial;
    t->nodes[id].pos = *pos;
    return id;
}

static int ct_best_edge(const ctree* t, const cnode* node) {
    const cedge* e = t->edges + node->first;
    int64_t sum = 0;
    for (int i = 0; i < node->count; ++i) sum += e[i].N;
    double sq = orc_pow_half(sum);
    int best = 0;
    double best_v = 0.0;
    for (int i = 0; i < node->count; ++i) {
        double q = e[i].N ? e[i].W / (double)e[i].N : 0.0;
        double u = t->c_puct * e[i].prior * sq / (double)(1 + e[i].N);
        double ucb = q + u;
        if (i == 0 || ucb > best_v) {
            best = i;
            best_v = ucb;
        }
    }
    return best;
}

static double ct_expand(ctree* t, int node_id) {
    float probs[ORC_CHESS_ACTIONS], value = 0.0f;
    cpos pos = t->nodes[node_id].pos;
    if (t->eval_kind == 0) {
        orc_chess_synth(&pos, t->nodes[node_id].initial, probs, &value);
    } else if (t->cb(t->ctx, &pos, t->nodes[node_id].initial, probs, &value) != 0) {
        t->error = 1;
    }
    uint16_t mv[256];
    int n = orc_chess_legal(&pos, mv);
    /* probabilities[legal_moves_mask]: legal actions in action order */
    int act[256];
    for (int i = 0; i < n; ++i) act[i] = action_index(mv[i]);
    float sorted[256];
    for (int i = 0; i < n; ++i) {
        int r = 0;
        for (int j = 0; j < n; ++j) r += act[j] < act[i];
        sorted[r] = probs[act[i]];
    }
    double priors[256];
    orc_normalize_f32(sorted, n, priors);
    if (t->n_edges + n > t->cap_edges) {
        while (t->n_edges + n > t->cap_edges) t->cap_edges = t->cap_edges ? 2 * t->cap_edges : 16384;
        t->edges = (cedge*)realloc(t->edges, sizeof(cedge) * (size_t)t->cap_edges);
    }
    int first = t->n_edges;
    for (int i = 0; i < n; ++i) {
        cpos child = pos;
        orc_chess_play_canonical(&child, mv[i]);
        int c = ct_new_node(t, &child, 0);
        cedge* e = t->edges + first + i;
        e->W = 0.0;
        e->prior = priors[i]; /* zip(probabilities, node.board.moves) */
        e->N = 0;
        e->child = c;
        e->action = mv[i];
    }
    t->n_edges += n;
    t->nodes[node_id].first = first;
    t->nodes[node_id].count = n;
    t->expansions++;
    return (double)value;
}

static void ct_search(ctree* t, int root, int sims) {
    int path[4096];
    for (int s = 0; s < sims; ++s) {
        int depth = 0, node = root;
        while (t->nodes[node].count) {
            int k = ct_best_edge(t, t->nodes + node);
            int e = t->nodes[node].first + k;
            if (depth < 4096) path[depth++] = e;
            node = t->edges[e].child;
        }
        double v;
        int oc = orc_chess_outcome(&t->nodes[node].pos);
        if (oc == 0) {
            v = -ct_expand(t, node);
        } else {
            v = oc == 1 ? 1.0 : 0.0;
            t->terminal_visits++;
        }
        for (int i = depth - 1; i >= 0; --i) {
            t->edges[path[i]].N += 1;
            t->edges[path[i]].W += v;
            v = -v;
        }
    }
}

/* MCTS.play's probabilities (mcts.py:188-196) and edge choice: np.argmax
 * when deterministic (mcts.py:198-199), else np.random.choice on the draw u
 * (cumsum, normalise by the last element, searchsorted right) */
static int ct_policy_choice(const ctree* t, const cnode* node, int greedy, int deterministic, double u,
                            double* pi) {
    int n = node->count;
    double counts[256];
    for (int i = 0; i < n; ++i) counts[i] = (double)t->edges[node->first + i].N;
    if (greedy) {
        int im = 0;
        for (int i = 1; i < n; ++i)
            if (counts[i] > counts[im]) im = i;
        for (int i = 0; i < n; ++i) pi[i] = i == im ? 1.0 : 0.0;
    } else {
        orc_normalize_f64(counts, n, pi);
    }
    if (deterministic) {
        int im = 0;
        for (int i = 1; i < n; ++i)
            if (pi[i] > pi[im]) im = i;
        return im;
    }
    double acc = 0.0, cdf[256];
    for (int i = 0; i < n; ++i) {
        acc += pi[i];
        cdf[i] = acc;
    }
    double last = cdf[n - 1];
    int idx = 0;
    for (int i = 0; i < n; ++i)
        if (cdf[i] / last <= u) idx = i + 1;
    return idx >= n ? n - 1 : idx;
}

typedef struct {
    int32_t T, result, termination;
    int64_t expansions, terminal_visits;
} orc_chess_game_out;

/* One chess self-play game.  Outputs per ply t < max_plies: positions[t]
 * (root before the move), moves[t], pol_n[t], pol_a[t][256] (action of each
 * root edge, edge order), pol_p[t][256] (MCTS.play probabilities), root
 * visit counts root_n[t][256]. */
int orc_chess_play_game(int sims, uint32_t seed, int max_plies, int greedy_ply, double c_puct,
                        int eval_kind,
                        int (*cb)(void*, const cpos*, int, float*, float*), void* ctx,
                        cpos* positions, uint16_t* moves, int32_t* pol_n, int16_t* pol_a,
                        double* pol_p, int64_t* root_visits, orc_chess_game_out* out) {
    init_tables();
    ctree t;
    memset(&t, 0, sizeof(t));
    t.c_puct = c_puct;
    t.eval_kind = eval_kind;
    t.cb = cb;
    t.ctx = ctx;
    orc_mt rng;
    orc_mt_seed(&rng, seed);
    cpos start;
    orc_chess_from_fen("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", &start);
    int root = ct_new_node(&t, &start, 1);
    int T = 0, term = 0;
    for (;;) {
        term = orc_chess_outcome(&t.nodes[root].pos);
        if (term != 0) break;
        if (T >= max_plies) {
            term = 5;
            break;
        }
        ct_search(&t, root, sims);
        cnode* node = t.nodes + root;
        int n = node->count;
        if (n == 0) {
            t.error = 1;
            break;
        }
        double pi[256];
        int idx = ct_policy_choice(&t, node, node->pos.fullmove_number >= greedy_ply, 0,
                                   orc_mt_uniform(&rng), pi);
        positions[T] = node->pos;
        moves[T] = t.edges[node->first + idx].action;
        pol_n[T] = n;
        for (int i = 0; i < n; ++i) {
            pol_a[(size_t)T * 256 + i] = (int16_t)action_index(t.edges[node->first + i].action);
            pol_p[(size_t)T * 256 + i] = pi[i];
            if (root_visits) root_visits[(size_t)T * 256 + i] = t.edges[node->first + i].N;
        }
        root = t.edges[node->first + idx].child;
        T++;
    }
    out->T = T;
    out->termination = term;
    out->result = term == 1 ? 1 : 0;
    out->expansions = t.expansions;
    out->terminal_visits = t.terminal_visits;
    int err = t.error;
    free(t.nodes);
    free(t.edges);
    return err ? -1 : 0;
}

/* ---------------------------------------------------------------------
 * One MCTS object (mcts.py:86-222) on a chess board, for the tree API
 * parity tests: the root node is marked initial (its board is a deepcopy,
 * history [0 x 7, start-position state]); play() moves the root to the
 * chosen child (tree reuse) and returns the new root's outcome.
 * ------------------------------------------------------------------- */
typedef struct {
    ctree t;
    int root;
} orc_chess_tree;

void* orc_chess_tree_new(const cpos* root, double c_puct, int eval_kind,
                         int (*cb)(void*, const cpos*, int, float*, float*), void* ctx) {
    init_tables();
    orc_chess_tree* h = (orc_chess_tree*)calloc(1, sizeof(orc_chess_tree));
    h->t.c_puct = c_puct;
    h->t.eval_kind = eval_kind;
    h->t.cb = cb;
    h->t.ctx = ctx;
    h->root = ct_new_node(&h->t, root, 1);
    return h;
}

void orc_chess_tree_search(void* hv, int sims) {
    orc_chess_tree* h = (orc_chess_tree*)hv;
    ct_search(&h->t, h->root, sims);
}

/* -> outcome of the new root (0 ongoing, 1..4), -1 when the root has no edges */
int orc_chess_tree_play(void* hv, double u, int greedy, int deterministic, uint16_t* move, int32_t* pol_n,
                        int16_t* pol_a, double* pol_p) {
    orc_chess_tree* h = (orc_chess_tree*)hv;
    cnode* node = h->t.nodes + h->root;
    int n = node->count;
    if (n == 0) return -1;
    double pi[256];
    int idx = ct_policy_choice(&h->t, node, greedy, deterministic, u, pi);
    *move = h->t.edges[node->first + idx].action;
    *pol_n = n;
    for (int i = 0; i < n; ++i) {
        pol_a[i] = (int16_t)action_index(h->t.edges[node->first + i].action);
        pol_p[i] = pi[i];
    }
    h->root = h->t.edges[node->first + idx].child;
    return orc_chess_outcome(&h->t.nodes[h->root].pos);
}

/* root edges in edge order: move, prior, N, W, and the child's edge count */
int orc_chess_tree_root(void* hv, uint16_t* moves, double* prior, int64_t* N, double* W, int32_t* child_n) {
    orc_chess_tree* h = (orc_chess_tree*)hv;
    const cnode* node = h->t.nodes + h->root;
    for (int i = 0; i < node->count; ++i) {
        const cedge* e = h->t.edges + node->first + i;
        moves[i] = e->action;
        prior[i] = e->prior;
        N[i] = e->N;
        W[i] = e->W;
        child_n[i] = h->t.nodes[e->child].count;
    }
    return node->count;
}

int64_t orc_chess_tree_expansions(void* hv) { return ((orc_chess_tree*)hv)->t.expansions; }

int orc_chess_tree_error(void* hv) { return ((orc_chess_tree*)hv)->t.error; }

void orc_chess_tree_free(void* hv) {
    orc_chess_tree* h = (orc_chess_tree*)hv;
    if (!h) return;
    free(h->t.nodes);
    free(h->t.edges);
    free(h);
}
