// az_chess.h -- chess rules on bitboards for the gfx950 kernels: python-chess
// 1.9.4's legal move generation (set AND order), push, mirror and outcome, as
// the reference's chess Board inherits them (custom_alphazero/chess/board.py).
//
// One thread owns one position.  Sliding attacks use per-direction ray
// tables (8 x 64 words, __constant__) and the first blocker's lsb/msb, so
// there is no magic-number table to stream through the caches; knight, king
// and pawn attacks are shifts.  The generation order is python-chess's
// (see oracle/chess_oracle.c for the restatement this must match bit for
// bit: tests/test_chess_gpu.py):
//   no check : pieces (not pawns) by from-square descending, to-squares
//              descending; castling (h-side rook first); pawn captures
//              (promotions Q, R, B, N); single pushes; double pushes; en passant
//   in check : king moves; captures/blocks of a single checker in the order
//              above; the en-passant capture of a checking pawn
//   then the _is_safe filter, which keeps the order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/az_chess.h"

// The rules compile for the host too (tests/native/chess_legal_check.cpp runs
// them under AddressSanitizer/UBSan against the oracle); the wave-parallel
// generators below are device-only (AZC_D).
#define AZC_HD __host__ __device__ __forceinline__
#define AZC_D __device__ __forceinline__

namespace azc {

typedef uint64_t bb;
enum { PAWN = 1, KNIGHT, BISHOP, ROOK, QUEEN, KING };
constexpr bb RANK_1 = 0xFFull, RANK_8 = 0xFF00000000000000ull;
constexpr bb FILE_A = 0x0101010101010101ull, FILE_H = 0x8080808080808080ull;
constexpr bb DARK = 0xAA55AA55AA55AA55ull;

// direction rays from each square, empty board, origin excluded.
// d: 0 N(+8) 1 NE(+9) 2 E(+1) 3 NW(+7) | 4 S(-8) 5 SW(-9) 6 W(-1) 7 SE(-7)
// (0-3 increase the square index: first blocker = lowest bit; 4-7: highest)
// Each translation unit that includes this header owns a copy and uploads it
// with upload_rays() once per device before its first launch.
static __constant__ bb c_rays[8][64];

static inline void host_rays(uint64_t rays[8][64]) {
  const int dirs[8][2] = {{0, 1}, {1, 1}, {1, 0}, {-1, 1}, {0, -1}, {-1, -1}, {-1, 0}, {1, -1}};
  for (int d = 0; d < 8; ++d)
    for (int s = 0; s < 64; ++s) {
      uint64_t r = 0;
      int f = (s & 7) + dirs[d][0], k = (s >> 3) + dirs[d][1];
      while (f >= 0 && f < 8 && k >= 0 && k < 8) {
        r |= 1ull << (k * 8 + f);
        f += dirs[d][0];
        k += dirs[d][1];
      }
      rays[d][s] = r;
    }
}
// the host copy (host builds of the rules)
static inline const uint64_t (*host_ray_table())[64] {
  static uint64_t rays[8][64];
  static bool init = false;
  if (!init) {
    host_rays(rays);
    init = true;
  }
  return rays;
}
AZC_HD bb ray_at(int d, int s) {
#ifdef __HIP_DEVICE_COMPILE__
  return c_rays[d][s];
#else
  return host_ray_table()[d][s];
#endif
}
// for the current device (hipSetDevice first)
static inline hipError_t upload_rays() {
  uint64_t rays[8][64];
  host_rays(rays);
  return hipMemcpyToSymbol(HIP_SYMBOL(c_rays), rays, sizeof(rays));
}

AZC_HD bb sq_bb(int s) { return 1ull << s; }
#ifdef __HIP_DEVICE_COMPILE__
AZC_HD int msb(bb x) { return 63 - __clzll(x); }
AZC_HD int lsb(bb x) { return __ffsll((long long)x) - 1; }
AZC_HD int popc(bb x) { return __popcll(x); }
#else  // host: the builtins, so UBSan reports a zero argument (no square)
AZC_HD int msb(bb x) { return 63 - __builtin_clzll(x); }
AZC_HD int lsb(bb x) { return __builtin_ctzll(x); }
AZC_HD int popc(bb x) { return __builtin_popcountll(x); }
#endif
AZC_HD bb bswap(bb x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((bb)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
}

AZC_HD bb ray_attack(int d, int s, bb occ) {
  bb a = ray_at(d, s);
  bb b = a & occ;
  if (b) a ^= ray_at(d, d < 4 ? lsb(b) : msb(b));
  return a;
}
AZC_HD bb rook_att(int s, bb occ) {
  return ray_attack(0, s, occ) | ray_attack(2, s, occ) | ray_attack(4, s, occ) | ray_attack(6, s, occ);
}
AZC_HD bb bishop_att(int s, bb occ) {
  return ray_attack(1, s, occ) | ray_attack(3, s, occ) | ray_attack(5, s, occ) | ray_attack(7, s, occ);
}
AZC_HD bb knight_att(int s) {
  bb b = sq_bb(s);
  bb l1 = (b >> 1) & 0x7F7F7F7F7F7F7F7Full, l2 = (b >> 2) & 0x3F3F3F3F3F3F3F3Full;
  bb r1 = (b << 1) & 0xFEFEFEFEFEFEFEFEull, r2 = (b << 2) & 0xFCFCFCFCFCFCFCFCull;
  bb h1 = l1 | r1, h2 = l2 | r2;
  return (h1 << 16) | (h1 >> 16) | (h2 << 8) | (h2 >> 8);
}
AZC_HD bb king_att(int s) {
  bb b = sq_bb(s);
  bb a = b | ((b << 1) & ~FILE_A) | ((b >> 1) & ~FILE_H);
  return (a | (a << 8) | (a >> 8)) & ~b;
}
// python-chess BB_PAWN_ATTACKS[color][s]
AZC_HD bb pawn_att(int color, int s) {
  bb b = sq_bb(s);
  return color ? (((b << 7) & ~FILE_H) | ((b << 9) & ~FILE_A))
               : (((b >> 7) & ~FILE_A) | ((b >> 9) & ~FILE_H));
}
// direction index from a to b, -1 if not on one line
AZC_HD int dir_of(int a, int b) {
  int df = (b & 7) - (a & 7), dr = (b >> 3) - (a >> 3);
  if (a == b || !(df == 0 || dr == 0 || df == dr || df == -dr)) return -1;
  int sf = (df > 0) - (df < 0), sr = (dr > 0) - (dr < 0);
  // (sf, sr) -> d
  if (sr > 0) return sf > 0 ? 1 : (sf == 0 ? 0 : 3);
  if (sr == 0) return sf > 0 ? 2 : 6;
  return sf > 0 ? 7 : (sf == 0 ? 4 : 5);
}
AZC_HD int opp_dir(int d) { return d ^ 4; }
// python-chess between(a, b): squares strictly between
AZC_HD bb between(int a, int b) {
  int d = dir_of(a, b);
  return d < 0 ? 0 : (ray_at(d, a) & ray_at(opp_dir(d), b));
}
// python-chess ray(a, b): the whole line through a and b
AZC_HD bb line(int a, int b) {
  int d = dir_of(a, b);
  return d < 0 ? 0 : (ray_at(d, a) | ray_at(opp_dir(d), a) | sq_bb(a));
}

struct Pos {
  bb p[6];      // pawns, knights, bishops, rooks, queens, kings
  bb co[2];     // [0] BLACK, [1] WHITE
  bb castling;  // rook squares
  int ep;       // -1 none
  int turn;     // 1 WHITE
  int rep;
  int half, full;

  AZC_HD bb occ() const { return co[0] | co[1]; }
  // colour / piece-type accessors by select: indexing co[] or p[] with a
  // runtime value put the whole Pos in scratch memory (104 B per lane)
  AZC_HD bb C(int c) const { return c ? co[1] : co[0]; }
  AZC_HD void C_or(int c, bb v) {
    if (c) co[1] |= v;
    else co[0] |= v;
  }
  AZC_HD void P_or(int type, bb v) {
    switch (type) {
      case 1: p[0] |= v; break;
      case 2: p[1] |= v; break;
      case 3: p[2] |= v; break;
      case 4: p[3] |= v; break;
      case 5: p[4] |= v; break;
      default: p[5] |= v; break;
    }
  }
};

AZC_HD Pos load_pos(const az_chess_pos& a) {
  Pos q;
#pragma unroll
  for (int i = 0; i < 6; ++i) q.p[i] = a.pieces[i];
  q.co[0] = a.occupied_co[0];
  q.co[1] = a.occupied_co[1];
  q.castling = a.castling_rights;
  q.ep = a.ep_square;
  q.turn = a.turn;
  q.rep = a.repetition;
  q.half = a.halfmove_clock;
  q.full = a.fullmove_number;
  return q;
}
AZC_HD void store_pos(const Pos& q, az_chess_pos& a) {
#pragma unroll
  for (int i = 0; i < 6; ++i) a.pieces[i] = q.p[i];
  a.occupied_co[0] = q.co[0];
  a.occupied_co[1] = q.co[1];
  a.castling_rights = q.castling;
  a.ep_square = (int16_t)q.ep;
  a.turn = (uint8_t)q.turn;
  a.repetition = (uint8_t)q.rep;
  a.halfmove_clock = (uint16_t)q.half;
  a.fullmove_number = (uint16_t)q.full;
}

AZC_HD int piece_at(const Pos& q, int s) {
  bb b = sq_bb(s);
#pragma unroll
  for (int t = 0; t < 6; ++t)
    if (q.p[t] & b) return t + 1;
  return 0;
}

// python-chess _attackers_mask(color, square, occupied)
AZC_HD bb attackers(const Pos& q, int color, int s, bb occ) {
  bb qr = q.p[QUEEN - 1] | q.p[ROOK - 1], qb = q.p[QUEEN - 1] | q.p[BISHOP - 1];
  bb a = (king_att(s) & q.p[KING - 1]) | (knight_att(s) & q.p[KNIGHT - 1]) |
         (pawn_att(!color, s) & q.p[PAWN - 1]);
  if (qr & q.C(color)) a |= rook_att(s, occ) & qr;
  if (qb & q.C(color)) a |= bishop_att(s, occ) & qb;
  return a & q.C(color);
}

AZC_HD int king_sq(const Pos& q, int color) {
  bb k = q.p[KING - 1] & q.C(color);
  return k ? msb(k) : -1;
}

// python-chess clean_castling_rights() (standard chess)
AZC_HD bb clean_castling(const Pos& q) {
  bb c = q.castling & q.p[ROOK - 1];
  bb w = c & RANK_1 & q.co[1] & (sq_bb(0) | sq_bb(7));
  bb b = c & RANK_8 & q.co[0] & (sq_bb(56) | sq_bb(63));
  if (!(q.co[1] & q.p[KING - 1] & sq_bb(4))) w = 0;
  if (!(q.co[0] & q.p[KING - 1] & sq_bb(60))) b = 0;
  return w | b;
}

// python-chess attacks_mask(square) of a non-pawn piece of the side to move
AZC_HD bb piece_attacks(const Pos& q, int s, bb occ) {
  bb b = sq_bb(s);
  if (b & q.p[KNIGHT - 1]) return knight_att(s);
  if (b & q.p[KING - 1]) return king_att(s);
  bb a = 0;
  if (b & (q.p[BISHOP - 1] | q.p[QUEEN - 1])) a |= bishop_att(s, occ);
  if (b & (q.p[ROOK - 1] | q.p[QUEEN - 1])) a |= rook_att(s, occ);
  return a;
}

// Move sink: the generator streams moves (in python-chess order) into `out`
struct MoveOut {
  uint16_t* m;
  int n;
  AZC_HD void add(int from, int to, int promo) {
    if (n < AZ_CHESS_MAX_MOVES) m[n] = (uint16_t)(from | (to << 6) | (promo << 12));
    n++;  // a count above AZ_CHESS_MAX_MOVES is reported as an error
  }
  AZC_HD void add_pawn(int from, int to) {
    int r = to >> 3;
    if (r == 0 || r == 7) {
      add(from, to, QUEEN);
      add(from, to, ROOK);
      add(from, to, BISHOP);
      add(from, to, KNIGHT);
    } else {
      add(from, to, 0);
    }
  }
};

AZC_HD bool attacked_for_king(const Pos& q, bb path, bb occ) {
  for (bb x = path; x; x &= ~sq_bb(msb(x)))
    if (attackers(q, !q.turn, msb(x), occ)) return true;
  return false;
}

AZC_HD void gen_castling(const Pos& q, bb from_mask, bb to_mask, MoveOut& o) {
  int t = q.turn;
  bb back = t ? RANK_1 : RANK_8;
  bb king = q.C(t) & q.p[KING - 1] & back & from_mask;
  king &= (~king + 1);
  if (!king) return;
  int ks = msb(king);
  bb occ = q.occ();
  int base = t ? 0 : 56;
  for (bb cand = clean_castling(q) & back & to_mask; cand; cand &= ~sq_bb(msb(cand))) {
    int rs = msb(cand);
    bb rook = sq_bb(rs);
    bool a_side = rook < king;
    int kto = base + (a_side ? 2 : 6), rto = base + (a_side ? 3 : 5);
    bb king_path = between(ks, kto), rook_path = between(rs, rto);
    if (!(((occ ^ king ^ rook) & (king_path | rook_path | sq_bb(kto) | sq_bb(rto))) ||
          attacked_for_king(q, king_path | king, occ ^ king) ||
          attacked_for_king(q, sq_bb(kto), occ ^ king ^ rook ^ sq_bb(rto))))
      o.add(ks, kto, 0);
  }
}

AZC_HD void gen_ep(const Pos& q, bb from_mask, bb to_mask, MoveOut& o) {
  int ep = q.ep;
  if (ep < 0 || !(sq_bb(ep) & to_mask) || (sq_bb(ep) & q.occ())) return;
  int t = q.turn;
  bb cap = q.p[PAWN - 1] & q.C(t) & from_mask & pawn_att(!t, ep) & (0xFFull << (8 * (t ? 4 : 3)));
  for (; cap; cap &= ~sq_bb(msb(cap))) o.add(msb(cap), ep, 0);
}

// python-chess generate_pseudo_legal_moves(from_mask, to_mask)
AZC_HD void gen_pseudo(const Pos& q, bb from_mask, bb to_mask, MoveOut& o) {
  int t = q.turn;
  bb own = q.C(t), occ = q.occ();
  for (bb np = own & ~q.p[PAWN - 1] & from_mask; np; np &= ~sq_bb(msb(np))) {
    int f = msb(np);
    for (bb mv = piece_attacks(q, f, occ) & ~own & to_mask; mv; mv &= ~sq_bb(msb(mv))) o.add(f, msb(mv), 0);
  }
  if (from_mask & q.p[KING - 1]) gen_castling(q, from_mask, to_mask, o);
  bb pawns = q.p[PAWN - 1] & own & from_mask;
  if (!pawns) return;
  for (bb c = pawns; c; c &= ~sq_bb(msb(c))) {
    int f = msb(c);
    for (bb tg = pawn_att(t, f) & q.C(!t) & to_mask; tg; tg &= ~sq_bb(msb(tg))) o.add_pawn(f, msb(tg));
  }
  bb single, dbl;
  if (t) {
    single = (pawns << 8) & ~occ;
    dbl = (single << 8) & ~occ & (0xFFull << 16 | 0xFFull << 24);
  } else {
    single = (pawns >> 8) & ~occ;
    dbl = (single >> 8) & ~occ & (0xFFull << 40 | 0xFFull << 32);
  }
  single &= to_mask;
  dbl &= to_mask;
  for (; single; single &= ~sq_bb(msb(single))) {
    int to = msb(single);
    o.add_pawn(to + (t ? -8 : 8), to);
  }
  for (; dbl; dbl &= ~sq_bb(msb(dbl))) {
    int to = msb(dbl);
    o.add(to + (t ? -16 : 16), to, 0);
  }
  if (q.ep >= 0) gen_ep(q, from_mask, to_mask, o);
}

AZC_HD bb slider_blockers(const Pos& q, int king) {
  bb rq = q.p[ROOK - 1] | q.p[QUEEN - 1], bq = q.p[BISHOP - 1] | q.p[QUEEN - 1];
  bb snipers = ((rook_att(king, 0) & rq) | (bishop_att(king, 0) & bq)) & q.C(!q.turn);
  bb blockers = 0, occ = q.occ();
  for (; snipers; snipers &= ~sq_bb(msb(snipers))) {
    bb b = between(king, msb(snipers)) & occ;
    if (b && sq_bb(msb(b)) == b) blockers |= b;
  }
  return blockers & q.C(q.turn);
}

// python-chess pin_mask(color, square): file, rank, then diagonal rays
AZC_HD bb pin_mask(const Pos& q, int color, int s) {
  int king = king_sq(q, color);
  if (king < 0) return ~0ull;
  bb sm = sq_bb(s), occ = q.occ();
  bb rq = q.p[ROOK - 1] | q.p[QUEEN - 1], bq = q.p[BISHOP - 1] | q.p[QUEEN - 1];
  bb empty_rook = rook_att(king, 0);
  bb rays[3] = {empty_rook & (FILE_A << (king & 7)), empty_rook & (RANK_1 << (8 * (king >> 3))),
                bishop_att(king, 0)};
  bb sl[3] = {rq, rq, bq};
  for (int i = 0; i < 3; ++i) {
    if (rays[i] & sm) {
      for (bb sn = rays[i] & sl[i] & q.C(!color); sn; sn &= ~sq_bb(msb(sn))) {
        int p = msb(sn);
        if ((between(p, king) & (occ | sm)) == sm) return line(king, p);
      }
      break;
    }
  }
  return ~0ull;
}

AZC_HD bool ep_skewered(const Pos& q, int king, int capturer) {
  int t = q.turn;
  int last_double = q.ep + (t ? -8 : 8);
  bb occ = (q.occ() & ~sq_bb(last_double) & ~sq_bb(capturer)) | sq_bb(q.ep);
  bb horiz = q.C(!t) & (q.p[ROOK - 1] | q.p[QUEEN - 1]);
  if ((ray_attack(2, king, occ) | ray_attack(6, king, occ)) & horiz) return true;
  bb diag = q.C(!t) & (q.p[BISHOP - 1] | q.p[QUEEN - 1]);
  return (bishop_att(king, occ) & diag) != 0;
}

AZC_HD bool is_safe(const Pos& q, int king, bb blockers, uint16_t m) {
  int from = m & 63, to = (m >> 6) & 63;
  if (from == king) {
    int diff = (from & 7) - (to & 7);
    if (diff > 1 || diff < -1) return true;  // castling
    return !attackers(q, !q.turn, to, q.occ());
  }
  int d = to - from;
  bool is_ep = q.ep == to && (q.p[PAWN - 1] & sq_bb(from)) && (d == 7 || d == 9 || d == -7 || d == -9) &&
               !(q.occ() & sq_bb(to));
  if (is_ep) return (pin_mask(q, q.turn, from) & sq_bb(to)) && !ep_skewered(q, king, from);
  return !(blockers & sq_bb(from)) || (line(from, to) & sq_bb(king));
}

// python-chess generate_legal_moves into out[0..AZ_CHESS_MAX_MOVES); returns
// the count (-1 if the pseudo-legal list would not fit); *check = the side to
// move is in check
AZC_HD int legal_moves(const Pos& q, uint16_t* out, bool* check) {
  MoveOut o{out, 0};
  int king = king_sq(q, q.turn);
  *check = false;
  if (king < 0) {
    gen_pseudo(q, ~0ull, ~0ull, o);
    return o.n > AZ_CHESS_MAX_MOVES ? -1 : o.n;
  }
  bb blockers = slider_blockers(q, king);
  bb checkers = attackers(q, !q.turn, king, q.occ());
  if (checkers) {
    *check = true;
    bb sliders = checkers & (q.p[BISHOP - 1] | q.p[ROOK - 1] | q.p[QUEEN - 1]);
    bb attacked = 0;
    for (bb s = sliders; s; s &= ~sq_bb(msb(s))) attacked |= line(king, msb(s)) & ~sq_bb(msb(s));
    for (bb mv = king_att(king) & ~q.C(q.turn) & ~attacked; mv; mv &= ~sq_bb(msb(mv))) o.add(king, msb(mv), 0);
    int checker = msb(checkers);
    if (sq_bb(checker) == checkers) {
      bb target = between(king, checker) | checkers;
      gen_pseudo(q, ~q.p[KING - 1], target, o);
      if (q.ep >= 0 && !(sq_bb(q.ep) & target) && q.ep + (q.turn ? -8 : 8) == checker)
        gen_ep(q, ~0ull, ~0ull, o);
    }
  } else {
    gen_pseudo(q, ~0ull, ~0ull, o);
  }
  if (o.n > AZ_CHESS_MAX_MOVES) return -1;
  int n = 0;
  for (int i = 0; i < o.n; ++i)
    if (is_safe(q, king, blockers, out[i])) out[n++] = out[i];
  return n;
}

// ---- wave-parallel generation: the 64 lanes of one wave (all active and
// converged) produce legal_moves' list in the same order, lane L owning
// square 63 - L (python-chess walks squares from the highest): per-lane
// counts, an exclusive prefix across the wave, then each lane writes its
// moves at its offset.  Candidates go to LDS (`cand`), the _is_safe filter
// runs one candidate per lane and compacts in order with a ballot.
AZC_D int wave_offset(int v, int lane, int* total) {
  int incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  *total = __shfl(incl, 63, 64);
  return incl - v;
}
AZC_D void wave_put(uint16_t* out, int k, int from, int to, int promo) {
  if (k < AZ_CHESS_MAX_MOVES) out[k] = (uint16_t)(from | (to << 6) | (promo << 12));
}
AZC_D int wave_put_pawn(uint16_t* out, int k, int from, int to) {
  const int r = to >> 3;
  if (r == 0 || r == 7) {
    wave_put(out, k, from, to, QUEEN);
    wave_put(out, k + 1, from, to, ROOK);
    wave_put(out, k + 2, from, to, BISHOP);
    wave_put(out, k + 3, from, to, KNIGHT);
    return k + 4;
  }
  wave_put(out, k, from, to, 0);
  return k + 1;
}
// a lane-0-only generator step (castling, en passant: at most two moves)
template <typename F>
AZC_D int wave_serial(uint16_t* out, int n, int lane, F&& gen) {
  int nn = n;
  if (lane == 0) {
    MoveOut o{out, n};
    gen(o);
    nn = o.n;
  }
  return __shfl(nn, 0, 64);
}

// gen_pseudo(from_mask, to_mask) appended at out[n..]; returns the new count
AZC_D int gen_pseudo_wave(const Pos& q, bb from_mask, bb to_mask, uint16_t* out, int n, int lane) {
  const int t = q.turn, sq = 63 - lane;
  const bb own = q.C(t), occ = q.occ();
  int total;
  {  // pieces other than pawns, from-square descending, targets descending
    const bb np = own & ~q.p[PAWN - 1] & from_mask;
    bb tg = ((np >> sq) & 1) ? piece_attacks(q, sq, occ) & ~own & to_mask : 0;
    int k = n + wave_offset(popc(tg), lane, &total);
    for (; tg; tg &= ~sq_bb(msb(tg))) wave_put(out, k++, sq, msb(tg), 0);
    n += total;
  }
  if (from_mask & q.p[KING - 1])
    n = wave_serial(out, n, lane, [&](MoveOut& o) { gen_castling(q, from_mask, to_mask, o); });
  const bb pawns = q.p[PAWN - 1] & own & from_mask;
  if (!pawns) return n;
  const bb promo = RANK_1 | RANK_8;
  {  // pawn captures, from-square descending (promotions Q, R, B, N)
    bb tg = ((pawns >> sq) & 1) ? pawn_att(t, sq) & q.C(!t) & to_mask : 0;
    int k = n + wave_offset(popc(tg & ~promo) + 4 * popc(tg & promo), lane, &total);
    for (; tg; tg &= ~sq_bb(msb(tg))) k = wave_put_pawn(out, k, sq, msb(tg));
    n += total;
  }
  bb single, dbl;
  if (t) {
    single = (pawns << 8) & ~occ;
    dbl = (single << 8) & ~occ & (0xFFull << 16 | 0xFFull << 24);
  } else {
    single = (pawns >> 8) & ~occ;
    dbl = (single >> 8) & ~occ & (0xFFull << 40 | 0xFFull << 32);
  }
  single &= to_mask;
  dbl &= to_mask;
  {  // single pushes, to-square descending
    const bool on = (single >> sq) & 1;
    const int k = n + wave_offset(on ? ((sq_bb(sq) & promo) ? 4 : 1) : 0, lane, &total);
    if (on) wave_put_pawn(out, k, sq + (t ? -8 : 8), sq);
    n += total;
  }
  {  // double pushes, to-square descending
    const bool on = (dbl >> sq) & 1;
    const int k = n + wave_offset(on ? 1 : 0, lane, &total);
    if (on) wave_put(out, k, sq + (t ? -16 : 16), sq, 0);
    n += total;
  }
  if (q.ep >= 0) n = wave_serial(out, n, lane, [&](MoveOut& o) { gen_ep(q, from_mask, to_mask, o); });
  return n;
}

// legal_moves with the wave: candidates in `cand` (LDS, AZ_CHESS_MAX_MOVES),
// the legal list in `out`; same return value and *check as legal_moves
AZC_D int legal_moves_wave(const Pos& q, uint16_t* cand, uint16_t* out, bool* check, int lane) {
  const int king = king_sq(q, q.turn);
  *check = false;
  int n = 0;
  if (king < 0) {
    n = gen_pseudo_wave(q, ~0ull, ~0ull, cand, 0, lane);
    if (n > AZ_CHESS_MAX_MOVES) return -1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int j = lane; j < n; j += 64) out[j] = cand[j];
    return n;
  }
  const bb blockers = slider_blockers(q, king);
  const bb checkers = attackers(q, !q.turn, king, q.occ());
  if (checkers) {
    *check = true;
    const bb sliders = checkers & (q.p[BISHOP - 1] | q.p[ROOK - 1] | q.p[QUEEN - 1]);
    bb attacked = 0;
    for (bb s = sliders; s; s &= ~sq_bb(msb(s))) attacked |= line(king, msb(s)) & ~sq_bb(msb(s));
    const bb kt = king_att(king) & ~q.C(q.turn) & ~attacked;  // king moves, targets descending
    const bool on = (kt >> (63 - lane)) & 1;
    int total;
    const int k = wave_offset(on ? 1 : 0, lane, &total);
    if (on) wave_put(cand, k, king, 63 - lane, 0);
    n = total;
    const int checker = msb(checkers);
    if (sq_bb(checker) == checkers) {
      const bb target = between(king, checker) | checkers;
      n = gen_pseudo_wave(q, ~q.p[KING - 1], target, cand, n, lane);
      if (q.ep >= 0 && !(sq_bb(q.ep) & target) && q.ep + (q.turn ? -8 : 8) == checker)
        n = wave_serial(cand, n, lane, [&](MoveOut& o) { gen_ep(q, ~0ull, ~0ull, o); });
    }
  } else {
    n = gen_pseudo_wave(q, ~0ull, ~0ull, cand, 0, lane);
  }
  if (n > AZ_CHESS_MAX_MOVES) return -1;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  int kept = 0;
  for (int base = 0; base < n; base += 64) {  // _is_safe, order kept
    const int j = base + lane;
    const uint16_t m = j < n ? cand[j] : 0;
    const bool keep = j < n && is_safe(q, king, blockers, m);
    const unsigned long long mask = __ballot(keep);
    if (keep) out[kept + __popcll(mask & ((1ull << lane) - 1ull))] = m;
    kept += __popcll(mask);
  }
  return kept;
}

AZC_HD void remove_piece(Pos& q, int s) {
  bb m = ~sq_bb(s);
#pragma unroll
  for (int t = 0; t < 6; ++t) q.p[t] &= m;
  q.co[0] &= m;
  q.co[1] &= m;
}
AZC_HD void set_piece(Pos& q, int s, int type, int color) {
  remove_piece(q, s);
  q.P_or(type, sq_bb(s));
  q.C_or(color, sq_bb(s));
}

// python-chess Board.push of a legal move (standard chess)
AZC_HD void push(Pos& q, uint16_t m) {
  int from = m & 63, to = (m >> 6) & 63, promo = m >> 12;
  int t = q.turn;
  int e = t ? 4 : 60;
  if (from == e && (q.p[KING - 1] & sq_bb(e))) {  // _to_chess960
    if (to == e + 2 && !(q.p[ROOK - 1] & sq_bb(e + 2))) to = e + 3;
    else if (to == e - 2 && !(q.p[ROOK - 1] & sq_bb(e - 2))) to = e - 4;
  }
  q.castling = clean_castling(q);
  int ep = q.ep;
  q.ep = -1;
  q.half++;
  if (!t) q.full++;
  bb from_bb = sq_bb(from), to_bb = sq_bb(to);
  bb touched = from_bb ^ to_bb;
  if ((touched & q.p[PAWN - 1]) || (touched & q.C(!t))) q.half = 0;
  int piece = piece_at(q, from);
  remove_piece(q, from);
  int captured = piece_at(q, to);
  q.castling &= ~to_bb & ~from_bb;
  if (piece == KING) q.castling &= ~(t ? RANK_1 : RANK_8);
  if (piece == PAWN) {
    int diff = to - from;
    if (diff == 16 && (from >> 3) == 1) q.ep = from + 8;
    else if (diff == -16 && (from >> 3) == 6) q.ep = from - 8;
    else if (to == ep && (diff == 7 || diff == 9 || diff == -7 || diff == -9) && !captured)
      remove_piece(q, ep + (t ? -8 : 8));
  }
  if (promo) piece = promo;
  if (piece == KING && (q.C(t) & to_bb)) {  // castling (king takes own rook)
    bool a_side = (to & 7) < (from & 7);
    remove_piece(q, from);
    remove_piece(q, to);
    int base = t ? 0 : 56;
    set_piece(q, base + (a_side ? 2 : 6), KING, t);
    set_piece(q, base + (a_side ? 3 : 5), ROOK, t);
  } else {
    set_piece(q, to, piece, t);
  }
  q.turn = !t;
  q.rep = 0;
}

// python-chess mirror(): flip_vertical, swap colours, flip turn; the copy
// drops the move stack (is_repetition() = False)
AZC_HD void mirror(Pos& q) {
#pragma unroll
  for (int t = 0; t < 6; ++t) q.p[t] = bswap(q.p[t]);
  bb w = bswap(q.co[1]), b = bswap(q.co[0]);
  q.co[1] = b;
  q.co[0] = w;
  q.castling = bswap(q.castling);
  if (q.ep >= 0) q.ep ^= 56;
  q.turn = !q.turn;
  q.rep = 0;
}

// Board.play(move, keep_same_player) (chess/board.py:162-173)
AZC_HD void play(Pos& q, uint16_t m, bool keep_same_player) {
  push(q, m);
  if (keep_same_player) {
    mirror(q);
    q.turn = 1;
  }
}

AZC_HD bool insufficient_color(const Pos& q, int c) {
  bb own = q.C(c), opp = q.C(!c);
  if (own & (q.p[PAWN - 1] | q.p[ROOK - 1] | q.p[QUEEN - 1])) return false;
  if (own & q.p[KNIGHT - 1]) return popc(own) <= 2 && !(opp & ~q.p[KING - 1] & ~q.p[QUEEN - 1]);
  if (own & q.p[BISHOP - 1]) {
    bb bi = q.p[BISHOP - 1];
    bool same = !(bi & DARK) || !(bi & ~DARK);
    return same && !q.p[PAWN - 1] && !q.p[KNIGHT - 1];
  }
  return true;
}

// python-chess outcome() termination given the legal move count and check flag
AZC_HD int outcome(const Pos& q, int n_legal, bool check) {
  if (check && n_legal == 0) return AZ_CHESS_CHECKMATE;
  if (insufficient_color(q, 0) && insufficient_color(q, 1)) return AZ_CHESS_INSUFFICIENT;
  if (n_legal == 0) return AZ_CHESS_STALEMATE;
  if (q.half >= 150) return AZ_CHESS_SEVENTYFIVE;
  return AZ_CHESS_ONGOING;
}

// Board.array code of square s as np.eye(13) indexes it: 0 empty, 1..6 white
// P..K, 13 + (-type) for black (chess/board.py:40-42, :114-125)
AZC_HD int onehot_index(const Pos& q, int s) {
  int t = piece_at(q, s);
  if (!t) return 0;
  return (q.co[1] & sq_bb(s)) ? t : 13 - t;
}

// chess.Board() (the start position)
AZC_HD Pos start_pos() {
  Pos q;
  q.p[0] = 0x00FF00000000FF00ull;  // pawns
  q.p[1] = 0x4200000000000042ull;  // knights
  q.p[2] = 0x2400000000000024ull;  // bishops
  q.p[3] = 0x8100000000000081ull;  // rooks
  q.p[4] = 0x0800000000000008ull;  // queens
  q.p[5] = 0x1000000000000010ull;  // kings
  q.co[1] = 0x000000000000FFFFull;
  q.co[0] = 0xFFFF000000000000ull;
  q.castling = 0x8100000000000081ull;
  q.ep = -1;
  q.turn = 1;
  q.rep = 0;
  q.half = 0;
  q.full = 1;
  return q;
}

// Board.full_state's per-board planes 112-117 (chess/board.py full_state):
// castling rights (own / opponent, queen- / king-side) and the move counters
AZC_HD void state_feats(const Pos& cur, float (&feat)[6]) {
  const bb c = clean_castling(cur);
  const bb back_t = cur.turn ? RANK_1 : RANK_8, back_o = cur.turn ? RANK_8 : RANK_1;
  feat[0] = (c & FILE_A & back_t) != 0;
  feat[1] = (c & FILE_H & back_t) != 0;
  feat[2] = (c & FILE_A & back_o) != 0;
  feat[3] = (c & FILE_H & back_o) != 0;
  feat[4] = (float)cur.full;
  feat[5] = (float)cur.half;
}

// planes k0..k0+3 (k0 >= 64) of network-input pixel pix of a board whose
// history is [0 x 6, start, cur] -- or [0 x 7, start-position state] for a
// root set by reset (`initial`) -- as encode_queue_kernel writes them: planes
// 84-97 the start position's one-hot (repetition plane 0), 98-111 the
// board's (its repetition count), 112-117 state_feats, the rest 0
AZC_HD void full_state4(const Pos& st, const Pos& cur, bool initial, const float (&feat)[6], int pix, int k0,
                        float (&v)[4]) {
  const int sq = (7 - (pix >> 3)) * 8 + (pix & 7);
  const int st_idx = onehot_index(st, sq), cur_idx = initial ? st_idx : onehot_index(cur, sq);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + i;
    float val = 0.f;
    if (k >= 112 && k < 118) val = feat[k - 112];
    else if (k >= 98 && k < 112)
      val = k - 98 == 13 ? (initial ? 0.f : (float)cur.rep) : (cur_idx == k - 98 ? 1.f : 0.f);
    else if (k >= 84 && k < 98 && !initial) val = k - 84 == 13 ? 0.f : (st_idx == k - 84 ? 1.f : 0.f);
    v[i] = val;
  }
}

// move -> action index (position in get_all_possible_moves), via the table
// [from][to][promo slot] built on the host (-1 = not an action)
AZC_HD int promo_slot(int promo) { return promo ? promo - 1 : 0; }  // 0, 1 N, 2 B, 3 R, 4 Q
AZC_HD int action_of(const int16_t* lut, uint16_t m) {
  return lut[((m & 63) * 64 + ((m >> 6) & 63)) * 5 + promo_slot(m >> 12)];
}

}  // namespace azc
