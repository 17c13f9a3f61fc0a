// az_device.h -- board rules, numerics and RNG shared by the gfx950 kernels
// and the engine's host code.  Every function here is a from-scratch
// restatement of a reference behaviour; each cites the reference line it
// must agree with bit for bit (parity: tests/test_engine_gpu.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AZ_HD __host__ __device__ __forceinline__

namespace az {

constexpr int kMaxCells = 128;    // boards up to 128 cells (two 64-bit words)
constexpr int kMaxActions = 128;  // action space (all_possible_moves) bound
constexpr int kNoChild = -1;

// ---------------------------------------------------------------- config
struct GameCfg {
  int H, W, HW, n, gravity, A;  // ConfigConnectN (reference config.py:38-47)
  int sims;                     // mcts_iterations (config.py:21)
  int greedy_ply;               // index_move_greedy (config.py:55)
  double c_puct;                // exploration_constant (config.py:51)
  int slots;                    // concurrent game slots on this device
  int arena_cap;                // halves == 1: edges per slot (a static arena per slot)
  int halves;                   // 2: pooled arenas with compaction (TreeDev::pool_*), else 1
  int max_depth;                // path buffer per slot (= HW)
  int pow_len;                  // entries of the pow(n, 0.5) table
  int noise;                    // ConfigMCTS.enable_dirichlet_noise (config.py:52): root Dirichlet noise
  double noise_alpha;           // dirichlet_noise_value (config.py:53)
  double noise_ratio;           // dirichlet_noise_ratio (config.py:54)
  int rng_skip;                 // MT19937 words a game's stream discards after seeding (az_config.rng_skip)
};

// Edge::action carries the action index in its low 14 bits; kPrior64 marks
// the edges of an expansion whose priors came from normalize_probabilities'
// float64 uniform branch (mcts/utils.py:13-14) -- the reference's noisy-prior
// arithmetic depends on the priors' dtype (mcts.py:72-76)
constexpr int kActMask = 0x3fff;
constexpr int kPrior64 = 0x4000;

// ----------------------------------------------------------------- board
// Canonical board: `own` = stones of the side to move (+1 in the reference's
// mirrored array, connect_n/board.py:244-246), `opp` = the other side (-1).
// Cell index y*W + x, row 0 = top row (the reference's array[0]).
struct Board {
  uint64_t own[2];
  uint64_t opp[2];
};

// word chosen by a select, not by indexing: a dynamically indexed two-word
// array is moved to LDS by the compiler (a ds_read per tested cell)
AZ_HD bool bit(const uint64_t m[2], int c) { return ((c < 64 ? m[0] : m[1]) >> (c & 63)) & 1ull; }
AZ_HD void set_bit(uint64_t m[2], int c) {
  const uint64_t v = 1ull << (c & 63);
  m[0] |= c < 64 ? v : 0ull;
  m[1] |= c < 64 ? 0ull : v;
}
AZ_HD bool empty_cell(const Board& b, int c) { return !bit(b.own, c) && !bit(b.opp, c); }

// Action index -> landing cell (or -1 if illegal).  Action order is
// get_all_possible_moves (board.py:130-146): column x with gravity, x-major
// product(range(W), range(H)) without.  Gravity landing row: board.py:211-225.
AZ_HD int action_cell(const GameCfg& g, const Board& b, int a) {
  if (g.gravity) {
    int row = -1;
    for (int y = 0; y < g.H; ++y) {
      if (!empty_cell(b, y * g.W + a)) break;
      row = y;
    }
    return row < 0 ? -1 : row * g.W + a;
  }
  const int x = a / g.H, y = a % g.H;
  const int c = y * g.W + x;
  return empty_cell(b, c) ? c : -1;
}

// Board.moves order (board.py:113-124): ascending column with gravity; the
// np.where row-major scan (y, then x) without.  Writes action indices.
AZ_HD int moves_order(const GameCfg& g, const Board& b, int* out) {
  int k = 0;
  if (g.gravity) {
    for (int x = 0; x < g.W; ++x)
      if (empty_cell(b, x)) out[k++] = x;
  } else {
    for (int y = 0; y < g.H; ++y)
      for (int x = 0; x < g.W; ++x)
        if (empty_cell(b, y * g.W + x)) out[k++] = x * g.H + y;
  }
  return k;
}

AZ_HD int count_moves(const GameCfg& g, const Board& b) {
  int k = 0;
  if (g.gravity) {
    for (int x = 0; x < g.W; ++x) k += empty_cell(b, x);
  } else {
    for (int c = 0; c < g.HW; ++c) k += empty_cell(b, c);
  }
  return k;
}

enum : int { kOngoing = 0, kWin = 1, kDraw = 2 };

// Board.play(move, keep_same_player=True) (board.py:233-250): push for the
// side to move, n-in-a-row through the new stone in the four directions of
// config.py:47 (board.py:178-204), draw when no move is left (:206-208),
// then mirror so the opponent becomes the side to move.
AZ_HD int play(const GameCfg& g, Board& b, int a) {
  const int c = action_cell(g, b, a);
  if (c < 0) return -1;
  set_bit(b.own, c);
  const int x0 = c % g.W, y0 = c / g.W;
  const int dirs[4][2] = {{0, 1}, {1, 1}, {1, 0}, {1, -1}};
  int status = kOngoing;
  for (int d = 0; d < 4 && status == kOngoing; ++d) {
    int count = 1;
    for (int s = 1; s >= -1 && status == kOngoing; s -= 2) {
      const int dx = dirs[d][0] * s, dy = dirs[d][1] * s;
      int x = x0 + dx, y = y0 + dy;
      while (x >= 0 && x < g.W && y >= 0 && y < g.H && bit(b.own, y * g.W + x)) {
        if (++count >= g.n) {
          status = kWin;
          break;
        }
        x += dx;
        y += dy;
      }
    }
  }
  if (status == kOngoing && count_moves(g, b) == 0) status = kDraw;
  Board m;
  m.own[0] = b.opp[0];
  m.own[1] = b.opp[1];
  m.opp[0] = b.own[0];
  m.opp[1] = b.own[1];
  b = m;
  return status;
}

// Board.play as bitboard arithmetic (the select descent's hot path): the same
// status and board as play() for every board the search reaches.  The win
// test runs over the whole board: a position the search plays from is never
// terminal, so the mover had no n-in-a-row before the stone, and any run
// after it passes through the new stone -- exactly play()'s test.  With
// gravity a column's empty cells are its top rows, so the landing row is the
// column's empty count minus one (action_cell's scan from the top).
struct M128 {
  uint64_t lo, hi;
};
AZ_HD M128 m_or(M128 a, M128 b) { return {a.lo | b.lo, a.hi | b.hi}; }
AZ_HD M128 m_and(M128 a, M128 b) { return {a.lo & b.lo, a.hi & b.hi}; }
AZ_HD M128 m_shl(M128 x, int k) {  // bit p + k of the result = bit p of x, 0 <= k < 128
  if (k == 0) return x;
  if (k >= 64) return {0ull, x.lo << (k - 64)};
  return {x.lo << k, (x.hi << k) | (x.lo >> (64 - k))};
}
AZ_HD M128 m_shr(M128 x, int k) {  // bit p of the result = bit p + k of x
  if (k == 0) return x;
  if (k >= 64) return {x.hi >> (k - 64), 0ull};
  return {(x.lo >> k) | (x.hi << (64 - k)), x.hi >> k};
}
AZ_HD int m_popc(M128 x) { return __builtin_popcountll(x.lo) + __builtin_popcountll(x.hi); }

// per-configuration masks: column 0, cells that start a run of n to the right
// (x <= W - n), cells that start one to the left (x >= n - 1), the top row
struct BoardMasks {
  M128 col0, left, right, top;
};
AZ_HD BoardMasks board_masks(const GameCfg& g) {
  BoardMasks mk{{0, 0}, {0, 0}, {0, 0}, {0, 0}};
  for (int y = 0; y < g.H; ++y) mk.col0 = m_or(mk.col0, m_shl({1ull, 0ull}, y * g.W));
  for (int x = 0; x < g.W; ++x) {
    const M128 cx = m_shl(mk.col0, x);
    if (x <= g.W - g.n) mk.left = m_or(mk.left, cx);
    if (x >= g.n - 1) mk.right = m_or(mk.right, cx);
    mk.top = m_or(mk.top, m_shl({1ull, 0ull}, x));
  }
  return mk;
}

AZ_HD bool m_run(M128 own, M128 start, int step, int n) {  // n stones from a start cell, stride step
  M128 m = m_and(own, start);
  for (int i = 1; i < n; ++i) {
    if (i * step >= kMaxCells) return false;  // the run would leave the 128 cells
    m = m_and(m, m_shr(own, i * step));
  }
  return (m.lo | m.hi) != 0;
}

AZ_HD int play_bb(const GameCfg& g, const BoardMasks& mk, Board& b, int a) {
  M128 occ{b.own[0] | b.opp[0], b.own[1] | b.opp[1]};
  int c;
  if (g.gravity) {
    const M128 col = m_shl(mk.col0, a);
    const int k = m_popc(m_and({~occ.lo, ~occ.hi}, col));
    if (k == 0) return -1;
    c = (k - 1) * g.W + a;
  } else {
    const int x = a / g.H, y = a % g.H;
    c = y * g.W + x;
    if (bit(b.own, c) || bit(b.opp, c)) return -1;
  }
  set_bit(b.own, c);
  const M128 own{b.own[0], b.own[1]};
  occ = m_or(occ, m_shl({1ull, 0ull}, c));
  const M128 all{~0ull, ~0ull};
  const bool win = m_run(own, mk.left, 1, g.n) || m_run(own, all, g.W, g.n) ||
                   m_run(own, mk.left, g.W + 1, g.n) || m_run(own, mk.right, g.W - 1, g.n);
  int status = kOngoing;
  if (win) {
    status = kWin;
  } else if (g.gravity ? ((~occ.lo & mk.top.lo) | (~occ.hi & mk.top.hi)) == 0 : m_popc(occ) == g.HW) {
    status = kDraw;
  }
  Board m;
  m.own[0] = b.opp[0];
  m.own[1] = b.opp[1];
  m.opp[0] = b.own[0];
  m.opp[1] = b.own[1];
  b = m;
  return status;
}

// play_bb for one gravity shape known at compile time whose cells fit one
// 64-bit word (Connect-4's 6x7: 42 cells) -- the select descent plays a move
// per tree level on every lane of the game's group, and play_bb's runtime
// n / W loops of 128-bit variable shifts cost ~1.7 us a level.
// Here every shift is a constant: a run of N through stride S is
// x & x>>S & x>>2S & ..., masked to the cells a run may start from (no
// wrap past the board edge; vertical runs past the last row read zeros).
// Same status and board as play() for every board the search reaches
// (tests/native/play_bb_check.cpp).
template <int H, int W>
constexpr uint64_t c64_col0() {
  uint64_t m = 0;
  for (int y = 0; y < H; ++y) m |= 1ull << (y * W);
  return m;
}
template <int H, int W, int lo, int hi>  // cells with lo <= x <= hi
constexpr uint64_t c64_cols() {
  uint64_t m = 0;
  for (int x = lo; x <= hi; ++x) m |= c64_col0<H, W>() << x;
  return m;
}
template <int S, int N>
AZ_HD uint64_t c64_run(uint64_t x) {  // bit p: cells p, p + S, ..., p + (N - 1) S all set
  uint64_t m = x;
#pragma unroll
  for (int i = 1; i < N; ++i) m &= x >> (i * S);
  return m;
}
template <int H, int W, int N>
AZ_HD int play_c64(Board& b, int a) {
  static_assert(H * W <= 64 && N >= 2 && N <= H && N <= W, "one-word gravity shapes");
  constexpr uint64_t col0 = c64_col0<H, W>();
  constexpr uint64_t left = c64_cols<H, W, 0, W - N>();      // a run to the right fits
  constexpr uint64_t right = c64_cols<H, W, N - 1, W - 1>();  // a run to the left fits
  constexpr uint64_t top = (1ull << W) - 1;
  const uint64_t own = b.own[0], opp = b.opp[0];
  const uint64_t occ = own | opp;
  const int k = __builtin_popcountll(~occ & (col0 << a));  // the column's empty cells: its top rows
  if (k == 0) return -1;
  const uint64_t stone = 1ull << ((k - 1) * W + a);
  const uint64_t mine = own | stone;
  const uint64_t win = (c64_run<1, N>(mine) & left) | c64_run<W, N>(mine) | (c64_run<W + 1, N>(mine) & left) |
                       (c64_run<W - 1, N>(mine) & right);
  const int status = win ? kWin : ((~(occ | stone) & top) == 0 ? kDraw : kOngoing);
  b.own[0] = opp;
  b.opp[0] = mine;  // (the high words stay 0: every cell is in word 0)
  return status;
}

// ---------------------------------------------------------------- numerics
// numpy float32 add.reduce = identity 0 + pairwise_sum (8 accumulators from
// n >= 8, 128-element blocks).  normalize_probabilities (mcts/utils.py:4-16)
// sums the masked network output this way.
AZ_HD float pairwise_sum_f32(const float* a, int n) {
  if (n < 8) {
    float r = 0.0f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  // n <= kMaxActions = 128: one pairwise block
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

AZ_HD double pairwise_sum_f64(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

// ------------------------------------------------------- synthetic evaluator
// oracle/synth.py, restated: dyadic priors k/64 and values k/128, one board
// in 64 with all-zero priors.  Used for bit-exact tree parity runs.
AZ_HD uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

AZ_HD uint64_t board_hash(const Board& b) {
  uint64_t h = splitmix64(b.own[0]);
  h = splitmix64(h ^ b.own[1]);
  h = splitmix64(h ^ b.opp[0]);
  return splitmix64(h ^ b.opp[1]);
}

AZ_HD void synth_eval(const Board& b, int A, float* probs, float* value) {
  const uint64_t h = board_hash(b);
  const uint64_t vh = splitmix64(h ^ 0x5555555555555555ull);
  *value = (float)(((double)(vh >> 56) - 128.0) / 128.0);
  if ((vh & 0x3F) == 0) {
    for (int a = 0; a < A; ++a) probs[a] = 0.0f;
    return;
  }
  uint64_t w = h;
  for (int a = 0; a < A; ++a) {
    if (a && a % 12 == 0) w = splitmix64(w);
    probs[a] = (float)((double)(((w >> (5 * (a % 12))) & 31) + 1) / 64.0);
  }
}

// --------------------------------------------------------------- MT19937
// Legacy np.random.seed / random_sample (init_genrand + 53-bit double from
// two outputs), one generator per game; state stored word-major [625][slots]
// so a wave touching the same word of 64 generators reads one line.
constexpr int kMtN = 624;

AZ_HD uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

}  // namespace az
