// az_tree.hip -- lockstep PUCT search over a forest of game trees on gfx950.
//
// One lane = one game slot.  Per simulation the engine launches
//   select  (PUCT descent, terminal backups, eval-queue compaction)
//   -> evaluator (network forward or synthetic) on the compacted queue
//   -> expand  (mask + normalise priors, allocate edges, backup).
// After `sims` simulations, `play` commits one move per slot.
//
// Arithmetic contract (bit-exact with the reference under numpy<2 legacy
// promotion):
//   UCB   = Q + U, Q = W/N or 0.0, U = ((1.5*prior)*pow(sumN,0.5))/(1+N), all
//           IEEE f64, no contraction (this file builds with -ffp-contract=off);
//           pow(sumN, 0.5) comes from a host-built libm table (mcts.py:50 is
//           Python `** 0.5`, i.e. libm pow, which differs from sqrt at 2921...)
//   best  = first maximum (np.argmax, mcts.py:64-68)
//   prior = float32 pairwise sum + float32 divide, or float64 1/n uniform
//   W    += v in path order leaf->root with v negated per level (mcts.py:163-168)
//   move  = cumsum / last / searchsorted-right on one legacy random_sample
#include "az_random.h"
#include "az_tree.h"

namespace az {

// threads per block of the per-game kernels (select / expand / play): 2
// waves, +1% games/s over 4 and 1 (a tree launch holds fewer of the CUs the
// other lane's tower needs than 1-wave blocks, less contention per CU than
// 4); 16 lanes: -3% (profiles/r3/game_block_ab_bench.txt,
// game_block128_ab_bench.txt).  The launch bound is the block size itself.
constexpr int kGameBlock = 128;

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ void stat_add(const TreeDev& t, int which, unsigned long long v) {
  atomicAdd(t.stats + which, v);
}

// Wave-aggregated counters.  Every game of a launch adds to the same few
// words (queue counts, stats); one atomic per wave instead of one per game
// keeps those words' L2 channel from serialising a launch's worth of
// same-address atomics.  Called by the lanes active at the call site (a
// divergent branch is fine: __ballot sees exactly those lanes).
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
// one unit per active lane: returns this lane's slot (base + rank among the active lanes)
__device__ __forceinline__ int wave_claim(int32_t* counter) {
  const unsigned long long m = __ballot(1);
  const int leader = __ffsll((long long)m) - 1;
  const int rank = __popcll(m & ((1ull << lane_id()) - 1));
  int base = 0;
  if (lane_id() == leader) base = atomicAdd(counter, __popcll(m));
  return __shfl(base, leader) + rank;
}
__device__ __forceinline__ unsigned long long wave_claim64(unsigned long long* counter) {
  const unsigned long long m = __ballot(1);
  const int leader = __ffsll((long long)m) - 1;
  const int rank = __popcll(m & ((1ull << lane_id()) - 1));
  unsigned long long base = 0;
  if (lane_id() == leader) base = atomicAdd(counter, (unsigned long long)__popcll(m));
  return __shfl(base, leader) + (unsigned long long)rank;
}
__device__ __forceinline__ void wave_count(int32_t* counter) {
  const unsigned long long m = __ballot(1);
  if (lane_id() == __ffsll((long long)m) - 1) atomicAdd(counter, __popcll(m));
}
// stats: the active lanes' v summed bit-slice by bit-slice (v < 2^8)
__device__ __forceinline__ void wave_stat(const TreeDev& t, int which, unsigned v = 1) {
  const unsigned long long m = __ballot(1);
  unsigned long long sum = 0;
#pragma unroll
  for (int bit = 0; bit < 8; ++bit) sum += (unsigned long long)__popcll(__ballot((v >> bit) & 1u)) << bit;
  if (lane_id() == __ffsll((long long)m) - 1 && sum) atomicAdd(t.stats + which, sum);
}
__device__ __forceinline__ void flag_error(const TreeDev& t, unsigned long long f) {
  atomicOr(t.stats + kStatErrors, f);
}

// MCTS.backup (mcts.py:163-168): N += 1, W += value along the path, the sign
// flipping per level.  A path's edges are distinct, so eight levels at a time
// issue their path and edge loads together instead of one dependent pair of
// round trips per level (the same additions, so the same bits).
__device__ __forceinline__ void backup(Edge* E, const int32_t* __restrict__ path, int depth, double v) {
  constexpr int K = 8;
  for (int d1 = depth; d1 > 0; d1 -= K) {
    int id[K], n[K];
    double w[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < d1) id[k] = path[d1 - 1 - k];
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < d1) {
        n[k] = E[id[k]].N;
        w[k] = E[id[k]].W;
      }
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < d1) {
        E[id[k]].N = n[k] + 1;
        E[id[k]].W = w[k] + v;
        v = -v;
      }
  }
}

// MT19937, state word-major: word w of slot g at mt[w * slots + g].
__device__ void mt_seed(const TreeDev& t, int slots, int g, uint32_t seed) {
  uint32_t prev = seed;
  t.mt[g] = seed;
  for (int i = 1; i < kMtN; ++i) {
    prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
    t.mt[(size_t)i * slots + g] = prev;
  }
  t.mt[(size_t)kMtN * slots + g] = kMtN;  // force a twist on first use
}

// One twist of a slot's state in place (m: its word 0, words `slots` apart),
// the serial loop's arithmetic in its order: word i takes words i, i+1 as
// they were and word i+397 (as it was below i = 227, already new from there
// on; word 0 is new when i = 623 reads it as i+1).  A batch of kTwistB words
// loads every operand before its first store -- none of a batch's loads reads
// a word that batch writes before that word's own update, and the words from
// earlier batches are stored ahead of them in program order -- so a twist is
// 39 memory round trips instead of 624 dependent load-store chains (a game's
// reset twists once: slot_reset).  Batches of 48 words (13 round trips)
// cost 3% of games/s (profiles/r6/ab_exp5.txt).
__device__ void mt_twist(uint32_t* m, size_t slots) {
  constexpr int kTwistB = 16;
  static_assert(kMtN % kTwistB == 0 && 227 >= kTwistB, "batches never read their own stores");
  uint32_t cur = m[0];
  for (int i0 = 0; i0 < kMtN; i0 += kTwistB) {
    uint32_t nx[kTwistB], far[kTwistB];
#pragma unroll
    for (int k = 0; k < kTwistB; ++k) {
      const int i = i0 + k;
      nx[k] = m[(size_t)(i + 1 < kMtN ? i + 1 : 0) * slots];
      far[k] = m[(size_t)(i + 397 < kMtN ? i + 397 : i - 227) * slots];
    }
#pragma unroll
    for (int k = 0; k < kTwistB; ++k) {
      const uint32_t y = (cur & 0x80000000u) | (nx[k] & 0x7fffffffu);
      m[(size_t)(i0 + k) * slots] = far[k] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      cur = nx[k];
    }
  }
}

__device__ uint32_t mt_next(const TreeDev& t, int slots, int g) {
  uint32_t* m = t.mt;
  uint32_t pos = m[(size_t)kMtN * slots + g];
  if (pos >= (uint32_t)kMtN) {
    mt_twist(m + g, (size_t)slots);
    pos = 0;
  }
  const uint32_t y = m[(size_t)pos * slots + g];
  m[(size_t)kMtN * slots + g] = pos + 1;
  return mt_temper(y);
}

// legacy random_sample: ((a >> 5) * 2^26 + (b >> 6)) / 2^53
__device__ double mt_uniform(const TreeDev& t, int slots, int g) {
  const uint32_t a = mt_next(t, slots, g) >> 5;
  const uint32_t b = mt_next(t, slots, g) >> 6;
  return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

__device__ void slot_reset(const GameCfg& g, const TreeDev& t, int s, int64_t gid,
                           uint32_t seed) {
  Board b;
  b.own[0] = b.own[1] = b.opp[0] = b.opp[1] = 0;
  t.root_board[s] = b;
  t.root_first[s] = 0;
  t.root_n[s] = 0;
  t.root_value[s] = 0.f;
  t.arena_top[s] = 0;
  if (g.halves > 1) {  // pooled: no chunk yet (the first expansion takes one)
    t.arena_end[s] = 0;
    t.slot_live[s] = 0;
  }
  t.ply[s] = 0;
  t.path_len[s] = 0;
  t.slot_expansions[s] = 0;
  t.game_id[s] = gid;
  t.last_move[s] = -1;
  t.last_status[s] = kOngoing;
  mt_seed(t, t.mt_stride, s, seed);
  // the reference's play_game draws np.random.rand(1, H, W, 4) building its
  // model between the seed and the game (az_config.rng_skip): the words are
  // skipped, not drawn -- a twist whenever the index runs out, then the index
  // (the state mt_next would leave, without 2 dependent round trips per word)
  if (g.rng_skip > 0) {
    uint32_t* m = t.mt + s;
    const size_t slots = (size_t)t.mt_stride;
    uint32_t pos = kMtN;  // mt_seed's
    for (int n = g.rng_skip; n > 0;) {
      if (pos >= (uint32_t)kMtN) {
        mt_twist(m, slots);
        pos = 0;
      }
      const int k = min(n, kMtN - (int)pos);
      pos += (uint32_t)k;
      n -= k;
    }
    m[(size_t)kMtN * slots] = pos;
  }
}

// ------------------------------------------------------------------- select
#ifdef AZ_SEL_STAMPS
// diagnostic build (profiles/sel_stamps.py): per-slot 100 MHz wall-clock
// stamps of the select phases, read back with az_diag_sel_stamps
__device__ unsigned long long g_sel_stamps[16384][12];
// (row: the slot's game_id address, unique across lanes for 16384 slots)
#define AZ_SEL_ROW(s) ((((uintptr_t)(t.game_id + (s))) >> 3) & 16383)
#define AZ_SEL_STAMP(s, k) (g_sel_stamps[AZ_SEL_ROW(s)][k] = wall_clock64())
#define AZ_SEL_VALUE(s, k, v) (g_sel_stamps[AZ_SEL_ROW(s)][k] = (unsigned long long)(v))
extern "C" int az_diag_sel_stamps(unsigned long long* out, int n_slots) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sel_stamps), (size_t)std::min(n_slots, 16384) * 96) == hipSuccess ? 0 : -1;
}
#else
#define AZ_SEL_STAMP(s, k) ((void)0)
#define AZ_SEL_VALUE(s, k, v) ((void)0)
#endif
// MCTS.select (mcts.py:111-120) + the terminal branch of MCTS.search
// (mcts.py:176-180).  Non-terminal leaves are appended to the eval queue.
__device__ __forceinline__ bool same_board(const Board& a, const Board& b) {
  return a.own[0] == b.own[0] && a.own[1] == b.own[1] && a.opp[0] == b.opp[0] &&
         a.opp[1] == b.opp[1];
}

// After the descent: the terminal branch of MCTS.search (mcts.py:176-180) or
// the plays_inferences probe and, on a miss, an evaluator row.  The slot's
// leaf record (leaf_src: this simulation's tag and where its outputs are;
// leaf_board) is what the expand launch reads, one thread per slot.
__device__ void leaf_tail(const GameCfg& g, const TreeDev& t, const CacheDev& c, int s, Edge* E,
                          const int32_t* path, int depth, int status, const Board& b) {
  wave_stat(t, kStatSims);
  wave_stat(t, kStatPathEdges, (unsigned)depth);
  AZ_SEL_STAMP(s, 3);
  if (depth > 0 && status != kOngoing) {
    // get_result(keep_same_player=True): 1 for the player who just moved, 0 draw
    backup(E, path, depth, status == kWin ? 1.0 : 0.0);
    wave_stat(t, kStatTerminal);
    return;
  }
  // the cache bucket's state words are requested before the queue claim's
  // atomic, so the two round trips overlap
  const uint64_t h = board_hash(b);
  uint32_t gen = 0, fp = 0, base = 0;
  uint32_t w[kCacheBucket];
  const uint64_t tag = (uint64_t)t.leaf_epoch << 32;
  t.leaf_board[s] = b;
  t.path_len[s] = depth;
  if (c.enabled) {
    gen = (uint32_t)__hip_atomic_load(c.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fp = cache_fp(h);
    base = cache_bucket(c, h);
#pragma unroll
    for (int k = 0; k < kCacheBucket; ++k)
      w[k] = __hip_atomic_load(c.state + base + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  AZ_SEL_STAMP(s, 4);
  if (!c.enabled) {  // every leaf evaluated: its queue position is its row
    const int q = wave_claim(t.eval_count);
    t.eval_board[q] = b;
    t.leaf_src[s] = tag | (uint32_t)(-(q + 1));
    wave_stat(t, kStatNNEvals);
    return;
  }
  // repr(board) in plays_inferences (mcts.py:123).  Entries may be published
  // concurrently by another lane's insert kernel: the acquire load pairs with
  // its release exchange, so a Ready entry's key and payload are complete
  // (a Claimed one reads as absent: the leaf is evaluated here, same result).
  // Every Ready entry is live (LRU eviction, az_tree.h).
  {
    // the board's bucket: kCacheBucket state words (one 64-B segment) read
    // at once with relaxed loads (above), scanned in registers; a candidate's
    // key is read after an acquire fence (pairs with the insert's release)
    int hit = -1;
    uint32_t hst = 0;
    // the fingerprint matches (inserts fill a bucket in slot order: nothing
    // past an empty slot), then ONE acquire for the wave -- a fence per
    // candidate position had the wave invalidating its CU's L1 (the tower
    // tiles' weight fragments too) up to 16 times -- then the keys in order
    uint32_t cm = 0;
    bool stop = false;
#pragma unroll
    for (int k = 0; k < kCacheBucket; ++k) {
      const uint32_t st = w[k];
      if (stop) continue;
      if (st == kCacheEmpty) stop = true;
      else if ((st & 3u) == kCacheReady && (st >> 16) == fp) cm |= 1u << k;
    }
    if (cm) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      for (; cm; cm &= cm - 1) {
        const int k = __builtin_ctz(cm);
        if (same_board(c.keys[base + k], b)) {
          hit = k;
#pragma unroll
          for (int kk = 0; kk < kCacheBucket; ++kk)
            if (kk == k) hst = w[kk];  // (constant indices: w stays in VGPRs)
          break;
        }
      }
    }
    bool use = hit >= 0;
    if (use && cache_age(hst, gen) != 0) {
      // a hit on an older generation moves the entry into the current one
      // (its last use: inserts evict the least recently used), at most one CAS
      // per entry per generation.  The CAS must win -- or find the entry
      // already moved by another reader and still this board -- else an insert
      // may be overwriting the slot and the board counts as a miss (az_tree.h)
      const uint32_t want = cache_word(fp, gen, kCacheReady);
      const uint32_t prev = atomicCAS(c.state + base + hit, hst, want);
      if (prev != hst) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        use = prev == want && same_board(c.keys[base + hit], b);
      }
    }
    if (use) {
      const uint32_t idx = base + hit;
      t.leaf_src[s] = tag | idx;
      AZ_SEL_STAMP(s, 5);
      AZ_SEL_VALUE(s, 7, depth | (1 << 16) | ((uint64_t)s << 32));
      wave_stat(t, kStatCacheHits);
      return;
    }
  }
  AZ_SEL_STAMP(s, 5);
  AZ_SEL_VALUE(s, 7, depth | (2 << 16) | ((uint64_t)s << 32));
  // miss: an evaluator row of its own.  (Rounds 2-6 shared one row between
  // the slots of a simulation that reached the same board -- a dedup table
  // and a last-block pass over its candidates; without them a board two
  // slots meet in one simulation is evaluated twice, the same outputs, so the
  // same searches; with the expand's per-slot leaf records +2.2%,
  // profiles/r6/ab_exp5.txt.)
  wave_count(t.miss_count);
  const int row = wave_claim(t.nn_count);
  t.nn_board[row] = b;
  t.leaf_src[s] = tag | (uint32_t)(-(row + 1));
  wave_stat(t, kStatNNEvals);
}

// ---------------------------------------------------- Dirichlet root noise
// get_best_edge_with_noise (mcts.py:70-85), used by select at the current
// root when ConfigMCTS.enable_dirichlet_noise is set (:113-116): a fresh
// np.random.dirichlet(alpha * ones(k)) per root selection -- in self-play
// from the game's MT19937 stream on the device (az_random.h), in the tree
// API drawn by the host from numpy's global stream (TreeDev::noise_in) --
// mixed into the priors as numpy computes
// (1 - ratio) * priors + ratio * noise -- the first product in the priors'
// dtype (float32, or float64 after the uniform branch: kPrior64), the rest
// float64 -- and the UCB with that prior; np.argmax treats NaN as the maximum.
struct SlotMt {  // the slot's MT19937 words, one at a time
  const TreeDev* t;
  int s;
  __device__ uint32_t operator()() { return mt_next(*t, t->mt_stride, s); }
};
__device__ __forceinline__ double noisy_prior(const GameCfg& g, const Edge& e, double d) {
  const double kept = (e.action & kPrior64) ? (1.0 - g.noise_ratio) * e.prior
                                            : (double)((float)(1.0 - g.noise_ratio) * (float)e.prior);
  return kept + g.noise_ratio * d;
}
// np.argmax order: NaN above every number, then value, then the lower index
__device__ __forceinline__ bool argmax_before(double v, int i, double bv, int bi) {
  if (bv != bv) return v != v && i < bi;
  if (v != v) return true;
  return v > bv || (v == bv && i < bi);
}

// Serial descent, one lane per game (used when the action space exceeds 64).
template <bool NOISE>
__device__ __forceinline__ void select_body(const GameCfg& g, const TreeDev& t, const CacheDev& c) {
  if (blockIdx.x == 0 && threadIdx.x < 4) t.next_counts[threadIdx.x * kCountStride] = 0;  // next simulation's counts
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.slots || t.game_id[s] < 0) return;
  const BoardMasks mk = board_masks(g);
  Edge* E = slot_edges(g, t, s);
  int32_t* path = t.path + (size_t)s * g.max_depth;
  Board b = t.root_board[s];
  int first = t.root_first[s], cnt = t.root_n[s];
  int depth = 0, status = kOngoing;
  while (cnt > 0) {
    int sum = 0;
    for (int i = 0; i < cnt; ++i) sum += E[first + i].N;
    if (sum >= g.pow_len) {
      flag_error(t, kErrPow);
      return;
    }
    const double sq = t.powtab[sum];
    int best = 0;
    double best_v = 0.0;
    if (NOISE && depth == 0) {
      double gam[kMaxActions], acc = 0.0;
      const double* hn = nullptr;  // tree API: the host's normalised draw
      if (t.noise_in) {
        const int row = t.noise_cur[s]++;
        if (row >= t.noise_rows) {
          flag_error(t, kErrNoise);
          return;
        }
        hn = t.noise_in + ((size_t)s * t.noise_rows + row) * g.A;
      } else {
        SlotMt r{&t, s};
        for (int i = 0; i < cnt; ++i) {
          gam[i] = legacy_standard_gamma(r, g.noise_alpha);
          acc = acc + gam[i];
        }
      }
      const double invacc = 1 / acc;
      for (int i = 0; i < cnt; ++i) {
        const Edge e = E[first + i];
        const double q = e.N ? e.W / (double)e.N : 0.0;
        const double u = g.c_puct * noisy_prior(g, e, hn ? hn[i] : gam[i] * invacc) * sq / (double)(1 + e.N);
        const double ucb = q + u;
        if (i == 0 || argmax_before(ucb, i, best_v, best)) {
          best = i;
          best_v = ucb;
        }
      }
    } else {
      for (int i = 0; i < cnt; ++i) {
        const Edge e = E[first + i];
        const double q = e.N ? e.W / (double)e.N : 0.0;
        const double u = g.c_puct * e.prior * sq / (double)(1 + e.N);
        const double ucb = q + u;
        if (i == 0 || ucb > best_v) {
          best = i;
          best_v = ucb;
        }
      }
    }
    if (depth >= g.max_depth) {
      flag_error(t, kErrPath);
      return;
    }
    const Edge& e = E[first + best];
    path[depth++] = first + best;
    status = play_bb(g, mk, b, e.action & kActMask);
    if (status < 0) {
      flag_error(t, kErrIllegal);
      return;
    }
    first = e.child;
    cnt = e.child_n;
  }
  leaf_tail(g, t, c, s, E, path, depth, status, b);
}

// Group descent: a game is a group of L lanes (L = next power of two >= A).
// Lane j loads edge j (contiguous, one 32-byte record per lane), the group
// sums N and takes the first-maximum UCB by shuffles -- the same float64
// expressions as the serial loop, so the chosen edge is identical.
// SHAPE 1: Connect-4 (6x7, n = 4, gravity) with the compile-time one-word
// play (play_c64); 0: any shape through play_bb's runtime masks.
template <int L, bool NOISE, int SHAPE>
__device__ __forceinline__ void select_group_body(const GameCfg& g, const TreeDev& t, const CacheDev& c) {
  if (blockIdx.x == 0 && threadIdx.x < 4) t.next_counts[threadIdx.x * kCountStride] = 0;  // next simulation's counts
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = gid / L, j = gid % L;
#ifdef AZ_SEL_STAMPS
  if (s < g.slots && j == 0) {
    AZ_SEL_STAMP(s, 0);
    for (int k = 1; k < 12; ++k) AZ_SEL_VALUE(s, k, 0);
  }
  // per-level phase sums (descent): edge data arrived, choice broadcast, play done
  unsigned long long ph_load = 0, ph_reduce = 0, ph_play = 0, ph_t = 0;
#define AZ_SEL_PHASE(acc)                   \
  do {                                      \
    __builtin_amdgcn_s_waitcnt(0);          \
    const unsigned long long now_ = wall_clock64(); \
    acc += now_ - ph_t;                     \
    ph_t = now_;                            \
  } while (0)
#else
#define AZ_SEL_PHASE(acc) ((void)0)
#endif
  if (s >= g.slots) return;  // whole groups leave together
  // the slot's game id and root read together (an idle slot's root is stale, unused)
  const int64_t game = t.game_id[s];
  Board b = t.root_board[s];
  int first = t.root_first[s], cnt = t.root_n[s];
  if (game < 0) return;
  if (j == 0) AZ_SEL_STAMP(s, 1);
  const BoardMasks mk = board_masks(g);
  Edge* E = slot_edges(g, t, s);
  int32_t* path = t.path + (size_t)s * g.max_depth;
  int depth = 0, status = kOngoing;
  // below the root, the children's visits sum to the parent edge's N - 1 (the
  // first visit expanded the node), so sqrt(sum) is fetched before the
  // children's edges arrive instead of after them: one dependent load per
  // level instead of two
  int sum_next = -1;
#ifdef AZ_SEL_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  if (j == 0) AZ_SEL_STAMP(s, 11);  // root loads done, loop entry
#endif
  while (cnt > 0) {
#ifdef AZ_SEL_STAMPS
    ph_t = wall_clock64();
#endif
    const bool mine = j < cnt;
    double sq;
    int sum;
    if (sum_next >= 0) {
      sum = sum_next;
      if (sum >= g.pow_len) {
        if (j == 0) flag_error(t, kErrPow);
        return;
      }
      sq = t.powtab[sum];
    }
    Edge e;
    if (mine) e = E[first + j];
    if (sum_next < 0) {
      sum = mine ? e.N : 0;
#pragma unroll
      for (int off = L / 2; off > 0; off >>= 1) sum += __shfl_xor(sum, off, L);
      if (sum >= g.pow_len) {
        if (j == 0) flag_error(t, kErrPow);
        return;
      }
      sq = t.powtab[sum];
    }
    AZ_SEL_PHASE(ph_load);
    double best_v = -INFINITY;
    int best = L;
    if (NOISE && depth == 0) {
      double dj = 0.0;  // this lane's edge's noise component
      if (t.noise_in) {
        // tree API: the host drew the vector from numpy's global stream
        int row = 0;
        if (j == 0) row = t.noise_cur[s]++;
        row = __shfl(row, 0, L);
        if (row >= t.noise_rows) {
          if (j == 0) flag_error(t, kErrNoise);
          return;
        }
        if (mine) dj = t.noise_in[((size_t)s * t.noise_rows + row) * g.A + j];
      } else {
        // the group walks the root's k gamma draws in order; its first lane
        // (the slot's RNG owner) draws, each lane keeps its edge's
        double acc = 0.0, gj = 0.0;
        for (int k = 0; k < cnt; ++k) {  // group-uniform
          double gv = 0.0;
          if (j == 0) {
            SlotMt r{&t, s};
            gv = legacy_standard_gamma(r, g.noise_alpha);
          }
          gv = __shfl(gv, 0, L);
          if (k == j) gj = gv;
          acc = acc + gv;
        }
        const double invacc = 1 / acc;
        dj = gj * invacc;
      }
      if (mine) {
        const double q = e.N ? e.W / (double)e.N : 0.0;
        const double u = g.c_puct * noisy_prior(g, e, dj) * sq / (double)(1 + e.N);
        best_v = q + u;
        best = j;
      }
#pragma unroll
      for (int off = L / 2; off > 0; off >>= 1) {
        const double ov = __shfl_xor(best_v, off, L);
        const int oj = __shfl_xor(best, off, L);
        if (argmax_before(ov, oj, best_v, best)) {
          best_v = ov;
          best = oj;
        }
      }
    } else {
      if (mine) {
        const double q = e.N ? e.W / (double)e.N : 0.0;
        const double u = g.c_puct * e.prior * sq / (double)(1 + e.N);
        best_v = q + u;
        best = j;
      }
#pragma unroll
      for (int off = L / 2; off > 0; off >>= 1) {
        const double ov = __shfl_xor(best_v, off, L);
        const int oj = __shfl_xor(best, off, L);
        if (ov > best_v || (ov == best_v && oj < best)) {  // np.argmax: first maximum
          best_v = ov;
          best = oj;
        }
      }
    }
    if (depth >= g.max_depth) {
      if (j == 0) flag_error(t, kErrPath);
      return;
    }
    const int action = __shfl(mine ? (int)(e.action & kActMask) : 0, best, L);
    const int child = __shfl(mine ? e.child : 0, best, L);
    const int child_n = __shfl(mine ? (int)e.child_n : 0, best, L);
    sum_next = __shfl(mine ? e.N : 0, best, L) - 1;
    AZ_SEL_PHASE(ph_reduce);
    if (j == 0) path[depth] = first + best;
    ++depth;
    if constexpr (SHAPE == 1) status = play_c64<6, 7, 4>(b, action);
    else status = play_bb(g, mk, b, action);
    AZ_SEL_PHASE(ph_play);
    if (status < 0) {
      if (j == 0) flag_error(t, kErrIllegal);
      return;
    }
    first = child;
    cnt = child_n;
  }
  if (j == 0) {
    AZ_SEL_STAMP(s, 2);
    AZ_SEL_VALUE(s, 8, ph_load);
    AZ_SEL_VALUE(s, 9, ph_reduce);
    AZ_SEL_VALUE(s, 10, ph_play);
    leaf_tail(g, t, c, s, E, path, depth, status, b);
    AZ_SEL_STAMP(s, 6);
  }
}

template <bool NOISE>
__global__ __launch_bounds__(kGameBlock) void select_kernel(GameCfg g, TreeDev t, CacheDev c) {
  select_body<NOISE>(g, t, c);
}
template <int L, bool NOISE, int SHAPE = 0>
__global__ __launch_bounds__(kGameBlock) void select_group_kernel(GameCfg g, TreeDev t, CacheDev c) {
  select_group_body<L, NOISE, SHAPE>(g, t, c);
}

// ------------------------------------------------------------ cache insert
// plays_inferences[repr(board)] = probabilities, value (mcts.py:142): one
// writer per distinct board (dedup), racing only for the bucket's first empty
// slot or its least recently used entry kCacheEvictAge+ generations old
// (az_tree.h); a lost race moves on to the next candidate.
// Called by every thread of an insert block (u: the thread's evaluator row;
// past the rows, no entry).  The entries' keys and payloads are published
// behind ONE release per block (every wave's stores drained, a barrier, lane
// 0's agent release, a barrier, then each thread's state word) instead of a
// full fence per wave (MI355X_MICROARCH.md, valid producer forms).
__device__ void cache_insert_row(const GameCfg& g, const TreeDev& t, const CacheDev& c,
                                 const float* __restrict__ probs, const float* __restrict__ values, int u) {
  const int rows = *t.nn_count;
  if ((u - (int)threadIdx.x) >= rows) return;  // block-uniform: the whole block past the rows
  int idx = -1;
  uint32_t word = 0;
  bool was_empty = false;
  if (u < rows) {
    const Board b = t.nn_board[u];
    const uint64_t h = board_hash(b);
    const uint32_t gen = (uint32_t)__hip_atomic_load(c.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t fp = cache_fp(h);
    const uint32_t base = cache_bucket(c, h);
    uint32_t w[kCacheBucket];
#pragma unroll
    for (int k = 0; k < kCacheBucket; ++k)
      w[k] = __hip_atomic_load(c.state + base + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t tried = 0;  // slots whose CAS lost (claimed or refreshed meanwhile)
    for (int attempt = 0; attempt < kCacheBucket && idx < 0; ++attempt) {
      // candidate: the first empty slot, else the oldest evictable entry (the
      // first of equal ages); scanned with constant indices (w stays in VGPRs)
      int pick = -1;
      uint32_t pst = 0, page = 0;
      bool pempty = false;
#pragma unroll
      for (int k = 0; k < kCacheBucket; ++k) {
        const uint32_t st = w[k];
        if (pempty || ((tried >> k) & 1u)) continue;
        if (st == kCacheEmpty) {
          pick = k, pst = st, pempty = true;
        } else if (c.gen_size) {
          const uint32_t age = cache_age(st, gen);
          if (age >= kCacheEvictAge && age > page) pick = k, pst = st, page = age;
        }
      }
      if (pick < 0) break;  // every entry of the bucket is in use: evaluated again when met
      if (atomicCAS(c.state + base + pick, pst, cache_word(fp, gen, kCacheClaimed)) == pst) {
        idx = (int)(base + pick);
        was_empty = pempty;
      } else {
        tried |= 1u << pick;
      }
    }
    if (idx >= 0) {
      c.keys[idx] = b;
      float* dst = c.pay + (size_t)idx * (g.A + 1);
      for (int a = 0; a < g.A; ++a) dst[a] = probs[(size_t)u * g.A + a];
      dst[g.A] = values[u];
      word = cache_word(fp, gen, kCacheReady);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (idx < 0) return;
  atomicExch(c.state + idx, word);
  wave_stat(t, kStatCacheInserts);
  if (was_empty) wave_claim64(c.ctl + 2);
  // every gen_size-th insert since the clear opens a new generation
  const unsigned long long n = wave_claim64(c.ctl + 1) + 1;
  if (c.gen_size && n % c.gen_size == 0) atomicAdd(c.ctl, 1ull);
}

// ------------------------------------------------------ synthetic evaluator
__global__ __launch_bounds__(256) void synth_eval_kernel(GameCfg g, const Board* __restrict__ boards,
                                                         const int32_t* __restrict__ count,
                                                         float* __restrict__ probs,
                                                         float* __restrict__ values) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *count) return;
  synth_eval(boards[i], g.A, probs + (size_t)i * g.A, values + i);
}

// ------------------------------------------------------------------- expand
// MCTS.evaluate_and_expand (mcts.py:145-161) with normalize_probabilities
// (mcts/utils.py:4-16), then backup(-value) (mcts.py:175, 163-168).
// With INSERT the same launch also publishes this simulation's evaluated
// boards to the cache (blocks from exp_blocks on, one nn row per thread):
// the entries the leaves expanded here read were stamped with the current
// generation by select, which an insert never evicts (kCacheEvictAge,
// az_tree.h), so the two halves are independent and share one launch.
// SHAPE 1 (Connect-4, 6x7, n = 4, gravity): the legal columns are the top
// row's empty cells, in action order = moves order, and fewer than 8 of them,
// so normalize's numpy sum is the plain left-to-right one -- no cell scans.
template <int MAXA, bool INSERT, int SHAPE = 0>
__global__ __launch_bounds__(kGameBlock) void expand_kernel(GameCfg g, TreeDev t, CacheDev c,
                                                     const float* __restrict__ probs,
                                                     const float* __restrict__ values, int exp_blocks) {
  if (INSERT && (int)blockIdx.x >= exp_blocks) {  // block-uniform
    cache_insert_row(g, t, c, probs, values, ((int)blockIdx.x - exp_blocks) * blockDim.x + threadIdx.x);
    return;
  }
  // one thread per slot, two round trips: 1. the slot's leaf record (this
  // simulation's tag: else no leaf to expand -- idle, terminal), arena and
  // path row; 2. the leaf's outputs and the path's edges -- each trip's loads
  // issued together (leaf records by slot, not a queue: one trip fewer)
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.slots) return;
  const uint64_t leaf = t.leaf_src[s];
  const Board b = t.leaf_board[s];
  Edge* E = slot_edges(g, t, s);
  const int top0 = t.arena_top[s];
  const int end0 = g.halves > 1 ? t.arena_end[s] : 0;
  const int live0 = g.halves > 1 ? t.slot_live[s] : 0;
  const int depth = t.path_len[s];
  const int exps = t.slot_expansions[s];
  const int32_t* path = t.path + (size_t)s * g.max_depth;
  constexpr int K = 8;  // path levels read ahead (deeper ones after, one batch at a time)
  int pv[K];
#pragma unroll
  for (int k = 0; k < K; ++k) pv[k] = k < g.max_depth ? path[k] : 0;
  if ((uint32_t)(leaf >> 32) != t.leaf_epoch) return;
  const int src = (int32_t)(uint32_t)leaf;
  const float* p;
  float v;
  if (src >= 0) {  // cache hit
    p = c.pay + (size_t)src * (g.A + 1);
    v = p[g.A];
  } else {
    const int row = -src - 1;
    p = probs + (size_t)row * g.A;
    v = values[row];
  }
  int pn[K];
  double pw[K];
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k < depth) {
      pn[k] = E[pv[k]].N;
      pw[k] = E[pv[k]].W;
    }
  float masked[MAXA];
  int moves[MAXA];
  int nl = 0, nm = 0;
  float sum = 0.0f;
  uint32_t legal = 0;
  if constexpr (SHAPE == 1) {
    static_assert(MAXA >= 7, "Connect-4 actions");
    legal = (uint32_t)(~(b.own[0] | b.opp[0])) & 0x7fu;  // columns with room
    float pa[7];
#pragma unroll
    for (int a = 0; a < 7; ++a) pa[a] = p[a];  // issued together
#pragma unroll
    for (int a = 0; a < 7; ++a)
      if ((legal >> a) & 1u) sum += pa[a];  // numpy pairwise_sum below 8 elements: 0 + a0 + a1 + ...
#pragma unroll
    for (int a = 0; a < 7; ++a) masked[a] = pa[a];
    nl = nm = __builtin_popcount(legal);
  } else {
    for (int a = 0; a < g.A; ++a)
      if (action_cell(g, b, a) >= 0) masked[nl++] = p[a];
    nm = moves_order(g, b, moves);
    sum = pairwise_sum_f32(masked, nl);
  }
  int first = top0;
  if (g.halves > 1) {
    // pooled arena: the run goes into the slot's current chunk, or a new one
    // of kPoolChunkA * A edges bumped off the lane's half (one atomic per wave)
    int end = end0;
    if (first + nm > end) {
      const int ch = kPoolChunkA * g.A;
      const unsigned long long m = __ballot(1);
      const int leader = __ffsll((long long)m) - 1;
      const int rank = __popcll(m & ((1ull << lane_id()) - 1));
      unsigned long long base = 0;
      if (lane_id() == leader) base = atomicAdd(t.pool_top, (unsigned long long)__popcll(m) * ch);
      base = __shfl(base, leader) + (unsigned long long)rank * ch;
      if (base + ch > (unsigned long long)t.pool_cap) {
        flag_error(t, kErrArena);
        return;
      }
      first = (int)base;
      end = first + ch;
      t.arena_end[s] = end;
    }
    t.slot_live[s] = live0 + nm;
  } else if (first + nm > g.arena_cap) {
    flag_error(t, kErrArena);
    return;
  }
  if constexpr (SHAPE == 1) {
    int k = 0;
#pragma unroll
    for (int a = 0; a < 7; ++a)
      if ((legal >> a) & 1u) {
        Edge e;
        e.W = 0.0;
        e.prior = sum == 0.0f ? 1.0 / (double)nl : (double)(masked[a] / sum);
        e.N = 0;
        e.child = kNoChild;
        e.child_n = 0;
        e.action = (int16_t)(a | (sum == 0.0f ? kPrior64 : 0));
        e.child_value = 0.f;
        E[first + k] = e;
        ++k;
      }
  } else {
    for (int k = 0; k < nm; ++k) {
      Edge e;
      e.W = 0.0;
      // zip(probabilities, board.moves) pairs priors (action order) with moves
      // (moves order) by position -- mcts.py:151; identical orders with gravity
      e.prior = sum == 0.0f ? 1.0 / (double)nl : (double)(masked[k] / sum);
      e.N = 0;
      e.child = kNoChild;
      e.child_n = 0;
      e.action = (int16_t)(moves[k] | (sum == 0.0f ? kPrior64 : 0));
      e.child_value = 0.f;
      E[first + k] = e;
    }
  }
  t.arena_top[s] = first + nm;
  if (depth == 0) {
    t.root_first[s] = first;
    t.root_n[s] = nm;
    t.root_value[s] = v;
  } else {
    int pe_id = 0;  // the leaf's edge: path[depth - 1]
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k == depth - 1) pe_id = pv[k];
    if (depth > K) pe_id = path[depth - 1];
    Edge& pe = E[pe_id];
    pe.child = first;
    pe.child_n = (int16_t)nm;
    pe.child_value = v;
  }
  // backup(-value) (mcts.py:175, 163-168): the edge at level d gets the
  // leaf's -value negated depth - 1 - d times -- each edge once, so the
  // levels' order does not change a bit
  const double vb = -(double)v;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k < depth) {
      E[pv[k]].N = pn[k] + 1;
      E[pv[k]].W = pw[k] + (((depth - 1 - k) & 1) ? -vb : vb);
    }
  if (depth > K) backup(E, path + K, depth - K, vb);  // levels K.. (rare): the leaf's edge gets vb
  t.slot_expansions[s] = exps + 1;
  wave_stat(t, kStatExpansions);
}

// --------------------------------------------------------------------- play
// MCTS.play (mcts.py:182-222) and the self_play.play_game move loop
// (self_play.py:59-67): greedy one-hot from fullmove_number >= index_move_greedy,
// else normalised visit counts; one uniform per move even when greedy.
template <int MAXA>
__global__ __launch_bounds__(kGameBlock) void play_kernel(GameCfg g, TreeDev t, SampleDev smp,
                                                   const double* __restrict__ uniforms,
                                                   int greedy_mode, int deterministic, int refill) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.slots || t.game_id[s] < 0) return;
  Edge* E = slot_edges(g, t, s);
  const int first = t.root_first[s], cnt = t.root_n[s];
  if (cnt <= 0) {
    flag_error(t, kErrNoRoot);
    return;
  }
  const int ply = t.ply[s];
  // greedy_mode < 0: self_play's rule fullmove_number >= index_move_greedy
  // (self_play.py:62); 0/1: the caller's MCTS.play(greedy=...) argument
  const bool greedy = greedy_mode < 0 ? ply >= g.greedy_ply : greedy_mode != 0;
  double pr[MAXA];
  if (greedy) {
    int best = 0;
    for (int i = 1; i < cnt; ++i)
      if (E[first + i].N > E[first + best].N) best = i;
    for (int i = 0; i < cnt; ++i) pr[i] = i == best ? 1.0 : 0.0;
  } else {
    double c[MAXA];
    for (int i = 0; i < cnt; ++i) c[i] = (double)E[first + i].N;
    const double sum = pairwise_sum_f64(c, cnt);
    for (int i = 0; i < cnt; ++i) pr[i] = sum == 0.0 ? 1.0 / (double)cnt : c[i] / sum;
  }
  int k;
  if (deterministic) {
    k = 0;
    for (int i = 1; i < cnt; ++i)
      if (pr[i] > pr[k]) k = i;
  } else {
    const double u = uniforms ? uniforms[s] : mt_uniform(t, t.mt_stride, s);
    double cdf[MAXA];
    double acc = 0.0;
    for (int i = 0; i < cnt; ++i) {
      acc += pr[i];
      cdf[i] = acc;
    }
    const double last = cdf[cnt - 1];
    k = 0;
    for (int i = 0; i < cnt; ++i)
      if (cdf[i] / last <= u) k = i + 1;
  }
  Edge chosen = E[first + k];
  chosen.action &= kActMask;
  double* lp = t.last_policy + (size_t)s * g.A;
  for (int a = 0; a < g.A; ++a) lp[a] = 0.0;
  for (int i = 0; i < cnt; ++i) lp[E[first + i].action & kActMask] = pr[i];
  const int64_t gid = t.game_id[s];
  const bool record = smp.n_games > 0 && gid >= smp.first_game && gid < smp.first_game + smp.n_games;
  if (record) {
    const size_t gi = (size_t)(gid - smp.first_game);
    const size_t si = gi * g.HW + ply;
    smp.boards[si] = t.root_board[s];
    smp.moves[si] = (int16_t)chosen.action;
    double* pol = smp.policy + si * g.A;
    for (int a = 0; a < g.A; ++a) pol[a] = lp[a];
  }
  Board b = t.root_board[s];
  const int status = play(g, b, chosen.action);
  t.root_board[s] = b;
  t.root_first[s] = chosen.child;
  t.root_n[s] = chosen.child_n;
  t.root_value[s] = chosen.child_value;
  t.ply[s] = ply + 1;
  t.last_move[s] = chosen.action;
  t.last_status[s] = status;
  stat_add(t, kStatPlies, 1);
  if (status == kOngoing) return;
  if (record) {
    const size_t gi = (size_t)(gid - smp.first_game);
    smp.length[gi] = ply + 1;
    smp.result[gi] = status == kWin ? 1 : 0;
    smp.expansions[gi] = t.slot_expansions[s];
    if (smp.done_ids) smp.done_ids[atomicAdd(smp.done_count, 1ull)] = gid;
  }
  stat_add(t, kStatGamesDone, 1);
  if (!refill) {
    t.game_id[s] = -1;
    return;
  }
  const unsigned long long nid = atomicAdd(t.stats + kStatNextGame, 1ull);
  if ((int64_t)nid < smp.first_game + smp.n_games)
    slot_reset(g, t, s, (int64_t)nid, (uint32_t)(smp.base_seed + (uint64_t)nid));
  else
    t.game_id[s] = -1;
}

// Tree reuse with reclamation (halves == 2), after play_kernel: the new
// root's subtree -- the nodes MCTS.play keeps by moving current_root to the
// chosen child (mcts.py:207) -- is copied into the lane's other pool half by
// a Cheney scan, one wave per slot: the root's edge run first, then for each
// scanned edge with an expanded child that child's run, placed by a
// prefix sum over the wave's 64 edges (BFS order; edges before `scan` point
// into the new half).  The destination is one bump of the slot's live edge
// count (a bound on the kept subtree); the next move's expansions fill its
// unused tail before taking chunks.  Everything else the game has left is
// dropped.  Edge values are copied bit for bit: the next search sees the same
// tree.
__global__ __launch_bounds__(64) void compact_kernel(GameCfg g, TreeDev t) {
  const int s = blockIdx.x, lane = threadIdx.x;
  if (t.game_id[s] < 0) return;
  const Edge* E = t.edges;
  const int first = t.root_first[s], n = t.root_n[s];
  if (n <= 0) {  // a fresh game (refilled slot) or a terminal root: nothing to keep
    if (lane == 0) {
      t.arena_top[s] = 0;
      t.arena_end[s] = 0;
      t.slot_live[s] = 0;
      t.root_first[s] = 0;
    }
    return;
  }
  const int need = t.slot_live[s];
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(t.dst_top, (unsigned long long)need);
  base = __shfl(base, 0);
  const bool room = base + (unsigned long long)need <= (unsigned long long)t.pool_cap;
  Edge* D = t.dst_edges + (room ? base : 0);
  int top = n, scan = 0;
  bool overflow = !room || n > need;
  if (!overflow) {
    for (int j = lane; j < n; j += 64) D[j] = E[first + j];
    __syncthreads();
  }
  while (!overflow && scan < top) {
    const int top0 = top;
    const int j = scan + lane;
    Edge e;
    int need_j = 0;
    if (j < top0) {
      e = D[j];
      if (e.child >= 0) need_j = e.child_n;
    }
    int incl = need_j;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    const int total = __shfl(incl, 63, 64);
    if (top0 + total > need) {
      overflow = true;
      break;
    }
    if (need_j) {
      const int nf = top0 + incl - need_j;
      for (int k = 0; k < need_j; ++k) D[nf + k] = E[e.child + k];
      e.child = (int)base + nf;  // a pool-half index
      D[j] = e;
    }
    top = top0 + total;
    scan = min(scan + 64, top0);
    __syncthreads();
  }
  if (lane == 0) {
    if (overflow) {
      flag_error(t, kErrArena);
      t.root_n[s] = 0;
      top = 0;
    }
    t.root_first[s] = (int)base;
    t.arena_top[s] = (int)base + top;
    t.arena_end[s] = overflow ? (int)base : (int)base + need;
    t.slot_live[s] = top;
    atomicMax(t.stats + kStatMaxRetained, (unsigned long long)top);
  }
}

// after a lane's compaction nothing lives in its current half: record how
// full it got and empty it (the host swaps the halves for the next move)
__global__ void pool_flip_kernel(TreeDev t) {
  if (threadIdx.x != 0) return;
  atomicMax(t.stats + kStatPoolHigh, *t.pool_top);
  *t.pool_top = 0;
}

// First n_first slots get games first_game .. first_game+n_first-1; the rest idle.
__global__ void slot_init_kernel(GameCfg g, TreeDev t, SampleDev smp, int64_t n_first) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.slots) return;
  if (s < n_first) {
    const int64_t gid = smp.first_game + s;
    slot_reset(g, t, s, gid, (uint32_t)(smp.base_seed + (uint64_t)gid));
  } else {
    t.game_id[s] = -1;
  }
}

// MCTS API: fresh tree on a given root board (the MCTS constructor,
// mcts.py:89-106), game id = slot index, no sample recording.
__global__ void slot_set_root_kernel(GameCfg g, TreeDev t, const int32_t* slots,
                                     const Board* boards, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = slots[i];
  slot_reset(g, t, s, s, 0u);
  t.root_board[s] = boards[i];
}

__global__ void slot_release_kernel(TreeDev t, const int32_t* slots, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) t.game_id[slots[i]] = -1;
}

// ------------------------------------------------------------ sample drain
// One workgroup per finished game: the game's record (drain_record_bytes)
// with its boards as int8 cells (+1 side to move, -1 opponent), the layout
// az_selfplay_results returns, so the host does no per-ply work.
size_t drain_record_bytes(const GameCfg& g) {
  const size_t b = 24 + (size_t)8 * g.HW * g.A + (size_t)2 * g.HW + (size_t)g.HW * g.HW;
  return (b + 15) & ~(size_t)15;
}

__global__ __launch_bounds__(256) void drain_pack_kernel(GameCfg g, SampleDev smp, int64_t from,
                                                         uint8_t* __restrict__ out, size_t rec) {
  const int i = blockIdx.x, tid = threadIdx.x;
  const int64_t gid = smp.done_ids[from + i];
  const size_t gi = (size_t)(gid - smp.first_game);
  uint8_t* r = out + (size_t)i * rec;
  const int T = smp.length[gi];
  if (tid == 0) {
    *reinterpret_cast<int64_t*>(r) = gid;
    int32_t* h = reinterpret_cast<int32_t*>(r + 8);
    h[0] = T;
    h[1] = smp.result[gi];
    h[2] = smp.expansions[gi];
    h[3] = 0;
  }
  double* pol = reinterpret_cast<double*>(r + 24);
  const double* src = smp.policy + gi * g.HW * g.A;
  for (int k = tid; k < g.HW * g.A; k += blockDim.x) pol[k] = k < T * g.A ? src[k] : 0.0;
  int16_t* mv = reinterpret_cast<int16_t*>(r + 24 + (size_t)8 * g.HW * g.A);
  for (int k = tid; k < g.HW; k += blockDim.x) mv[k] = k < T ? smp.moves[gi * g.HW + k] : (int16_t)0;
  int8_t* cells = reinterpret_cast<int8_t*>(mv + g.HW);
  for (int k = tid; k < g.HW * g.HW; k += blockDim.x) {
    const int p = k / g.HW, c = k - p * g.HW;
    int8_t v = 0;
    if (p < T) {
      const Board& b = smp.boards[gi * g.HW + p];
      v = bit(b.own, c) ? 1 : (bit(b.opp, c) ? -1 : 0);
    }
    cells[k] = v;
  }
}

void launch_drain_pack(const GameCfg& g, const SampleDev& smp, int64_t from, int n, uint8_t* out,
                       hipStream_t s) {
  if (n > 0) drain_pack_kernel<<<n, 256, 0, s>>>(g, smp, from, out, drain_record_bytes(g));
}

// ---------------------------------------------------------------- launchers
static inline int blocks_for(int n) { return (n + 255) / 256; }
static inline int game_blocks(int n) { return (n + kGameBlock - 1) / kGameBlock; }

void launch_select(const GameCfg& g, const TreeDev& t, const CacheDev& c, hipStream_t s) {
  const int lanes = g.A <= 8 ? 8 : g.A <= 16 ? 16 : g.A <= 32 ? 32 : g.A <= 64 ? 64 : 1;
  const int blocks = (int)(((int64_t)g.slots * lanes + kGameBlock - 1) / kGameBlock);
  const bool c4 = g.H == 6 && g.W == 7 && g.n == 4 && g.gravity && lanes == 8;
  if (c4) {  // Connect-4: the compile-time one-word play (play_c64)
    if (g.noise) select_group_kernel<8, true, 1><<<blocks, kGameBlock, 0, s>>>(g, t, c);
    else select_group_kernel<8, false, 1><<<blocks, kGameBlock, 0, s>>>(g, t, c);
    return;
  }
  if (g.noise) {  // the root-noise instantiations (the default path carries none of their code)
    switch (lanes) {
      case 8: select_group_kernel<8, true><<<blocks, kGameBlock, 0, s>>>(g, t, c); break;
      case 16: select_group_kernel<16, true><<<blocks, kGameBlock, 0, s>>>(g, t, c); break;
      case 32: select_group_kernel<32, true><<<blocks, kGameBlock, 0, s>>>(g, t, c); break;
      case 64: select_group_kernel<64, true><<<blocks, kGameBlock, 0, s>>>(g, t, c); break;
      default: select_kernel<true><<<game_blocks(g.slots), kGameBlock, 0, s>>>(g, t, c); break;
    }
    return;
  }
  switch (lanes) {
    case 8: select_group_kernel<8, false><<<blocks, kGameBlock, 0, s>>>(g, t, c); break;
    case 16: select_group_kernel<16, false><<<blocks, kGameBlock, 0, s>>>(g, t, c); break;
    case 32: select_group_kernel<32, false><<<blocks, kGameBlock, 0, s>>>(g, t, c); break;
    case 64: select_group_kernel<64, false><<<blocks, kGameBlock, 0, s>>>(g, t, c); break;
    default: select_kernel<false><<<game_blocks(g.slots), kGameBlock, 0, s>>>(g, t, c); break;
  }
}

void launch_synth_eval(const GameCfg& g, const Board* boards, const int32_t* count, float* probs,
                       float* values, hipStream_t s) {
  synth_eval_kernel<<<blocks_for(g.slots), 256, 0, s>>>(g, boards, count, probs, values);
}

void launch_expand(const GameCfg& g, const TreeDev& t, const CacheDev& c, const float* probs,
                   const float* values, hipStream_t s) {
  const int eb = game_blocks(g.slots);
  const bool ins = c.enabled;
  const int grid = eb + (ins ? game_blocks(g.slots) : 0);
  if (g.H == 6 && g.W == 7 && g.n == 4 && g.gravity) {  // Connect-4: the top-row form
    if (ins) expand_kernel<16, true, 1><<<grid, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);
    else expand_kernel<16, false, 1><<<grid, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);
  } else if (g.A <= 16) {
    if (ins) expand_kernel<16, true><<<grid, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);
    else expand_kernel<16, false><<<grid, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);
  } else {
    if (ins) expand_kernel<kMaxActions, true><<<grid, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);
    else expand_kernel<kMaxActions, false><<<grid, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);
  }
}

void launch_play(const GameCfg& g, const TreeDev& t, const SampleDev& smp, const double* uniforms,
                 int greedy_mode, int deterministic, int refill, hipStream_t s) {
  if (g.A <= 16)
    play_kernel<16><<<game_blocks(g.slots), kGameBlock, 0, s>>>(g, t, smp, uniforms, greedy_mode,
                                                                deterministic, refill);
  else
    play_kernel<kMaxActions><<<game_blocks(g.slots), kGameBlock, 0, s>>>(
        g, t, smp, uniforms, greedy_mode, deterministic, refill);
}

void launch_compact(const GameCfg& g, const TreeDev& t, hipStream_t s) {
  if (g.halves <= 1) return;
  if (g.slots > 0) compact_kernel<<<g.slots, 64, 0, s>>>(g, t);
  pool_flip_kernel<<<1, 64, 0, s>>>(t);
}

// Every lane's play kernel for move m + 1 waits for the other lanes' move m
// (az_engine.hip), so when the last lane arrives here no game of move m + 1
// has been appended: done_count is exactly the games finished by move m.
__global__ void move_end_kernel(int32_t* arrive, int n_lanes, const unsigned long long* done_count,
                                unsigned long long* snap) {
  if (threadIdx.x != 0) return;
  const int prev = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (prev != n_lanes - 1) return;
  __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long d = __hip_atomic_load(done_count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(snap, d, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_move_end(int32_t* arrive, int n_lanes, const unsigned long long* done_count,
                     unsigned long long* snap, hipStream_t s) {
  move_end_kernel<<<1, 64, 0, s>>>(arrive, n_lanes, done_count, snap);
}

void launch_slot_init(const GameCfg& g, const TreeDev& t, const SampleDev& smp, int64_t n_first,
                      hipStream_t s) {
  slot_init_kernel<<<blocks_for(g.slots), 256, 0, s>>>(g, t, smp, n_first);
}

void launch_slot_release(const TreeDev& t, const int32_t* slots, int n, hipStream_t s) {
  if (n > 0) slot_release_kernel<<<(n + 255) / 256, 256, 0, s>>>(t, slots, n);
}

void launch_slot_set_root(const GameCfg& g, const TreeDev& t, const int32_t* slots,
                          const Board* boards, int n, hipStream_t s) {
  if (n > 0) slot_set_root_kernel<<<blocks_for(n), 256, 0, s>>>(g, t, slots, boards, n);
}

}  // namespace az
