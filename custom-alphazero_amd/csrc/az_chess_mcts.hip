// az_chess_mcts.hip -- chess self-play on gfx950 (BASELINE configs[4]):
// the MCTS of custom_alphazero/mcts/mcts.py over the chess rules of
// az_chess.h, with the policy/value network of az_nn.hip on 118-plane states.
//
// One simulation for every game slot per step, as in the Connect-N engine
// (az_tree.hip), but a chess node has up to 218 edges and a game has no fixed
// length, so:
//   select   one wave per slot: PUCT over the node's edges (4 per lane),
//            ΣN and first-max argmax by wave shuffles, the position replayed
//            along the path with push + mirror (no boards stored per node)
//   leaf     one wave per slot: legal moves (one square per lane) + outcome of
//            the leaf; terminal leaves back up get_result's value, the rest
//            join the eval queue
//   encode   one workgroup per queued board: Board.full_state planes straight
//            into the network input (padded to 128 channels)
//   expand   one wave per queued board: priors = probs[mask] renormalised in
//            action order (float32 pairwise sum) and zipped positionally with
//            python-chess's move order (mcts.py:147-160), edges allocated, backup
//   play     one wave per slot: MCTS.play policy + np.random.choice, sample
//            record, and the chosen child's subtree copied (Cheney scan) into
//            the other half of the slot's edge arena (tree reuse,
//            mcts.py:212), then the new root's game-over check and slot refill.
// Arithmetic contract as az_tree.hip (this file builds with -ffp-contract=off).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/az_chess.h"
#include "az_chess.h"
#include "az_nn.h"
#include "az_tree.h"

namespace az {
int fail_abi(int code, const std::string& msg);
}

namespace azc {
std::vector<int16_t> action_lut();  // az_chess.hip

namespace {

using az::Edge;

struct CCfg {
  int slots, sims, greedy_ply, half_cap, max_depth, max_plies, pow_len, evaluator;
  double c_puct;
};

struct CTree {
  Edge* edges;             // [slots][2][half_cap]
  az_chess_pos* root;      // [slots]
  int32_t* root_first;     // [slots]
  int32_t* root_n;         // [slots]
  int32_t* half;           // [slots] arena half holding the live tree
  int32_t* top;            // [slots] edges used in that half
  int32_t* ply;            // [slots]
  int32_t* initial;        // [slots] root is the game's Board() (history [0 x 7, state])
  int64_t* game_id;        // [slots], -1 idle
  int32_t* path;           // [slots][max_depth]
  int32_t* path_len;       // [slots]
  az_chess_pos* leaf;      // [slots]
  uint16_t* leaf_moves;    // [slots][AZ_CHESS_MAX_MOVES]
  int32_t* leaf_n;         // [slots]
  int32_t* slot_exp;       // [slots]
  float* root_value;       // [slots] the root's evaluated_value (tree API views)
  uint32_t* mt;            // [625][mt_stride] word-major MT19937 (a lane view offsets it)
  int32_t mt_stride;       // slots of the whole engine
  int32_t* eval_slot;      // [slots]
  int32_t* eval_count;     // this simulation's queue length (one of the lane's two counters)
  int32_t* next_count;     // the other: zeroed by this simulation's select launch for the next one
  int32_t* slot_q;         // [slots] the slot's leaf in its last simulation (the fused expand): its
                           // network row (>= 0), kQHit (served by the transposition cache: the
                           // payload copied to leaf_pay), -1 none; kQDup0 - k while a duplicate waits
                           // for the launch's last block (tag slot k of the dedup table)
  unsigned long long* stats;
  const double* powtab;
  const int16_t* lut;
  // transposition cache (round 6; null when off) = the reference's
  // plays_inferences for chess boards (mcts.py:122-143): key = the leaf
  // position + its history form (the network input is a function of both),
  // payload = the masked, action-ordered network priors (normalize's input)
  // and the value.  Per-simulation dedup of identical leaves (step table,
  // epoch-tagged) gives duplicates the owner's network row.
  float* leaf_pay;         // [slots][kPayFloats] a hit's payload, copied in the select launch
  uint64_t* step_tag;      // [step_mask + 1] (epoch << 32) | fingerprint
  int32_t* step_row;       // [step_mask + 1] the owner's network row
  uint32_t step_mask;
  uint32_t epoch;
  int32_t* dup_q;          // [slots] duplicate slots of this simulation
  int32_t* dup_count;      // this simulation's (the lane's counts block, alternating)
  int32_t* next_dup;       // the next simulation's (zeroed by this select launch)
  uint32_t* sel_done;      // [1] select blocks finished (the last resolves the duplicates)
};

constexpr int kQHit = -2, kQDup0 = -3;
// transposition cache entry: key (position + history form), state word, payload
struct ChessKey {
  az_chess_pos pos;  // 80 B
  int32_t initial;   // the root's [0 x 7, start] history form (see encode_queue_kernel)
  int32_t pad[3];
};
static_assert(sizeof(ChessKey) == 96, "ChessKey is 6 uint4");
constexpr int kPayFloats = AZ_CHESS_MAX_MOVES + 4;  // priors in action order [n], then value at [256]
struct ChessCache {
  ChessKey* keys = nullptr;      // [cap]
  uint32_t* state = nullptr;     // [cap] az_tree.h cache_word (fingerprint, generation, status)
  float* pay = nullptr;          // [cap][kPayFloats]
  uint32_t mask = 0;
  int enabled = 0;
  unsigned long long* ctl = nullptr;  // [0] generation, [1] inserts since the clear, [2] into empty slots
  unsigned long long gen_size = 0;
};

struct CSamples {
  int64_t first_game = 0, n_games = 0;
  uint32_t base_seed = 0;
  int plies = 0;
  az_chess_pos* pos = nullptr;   // [G][P]
  uint16_t* moves = nullptr;     // [G][P]
  int32_t* pol_n = nullptr;      // [G][P]
  int16_t* pol_a = nullptr;      // [G][P][256]
  double* pol_p = nullptr;       // [G][P][256]
  int32_t* length = nullptr;     // [G]
  int32_t* result = nullptr;
  int32_t* term = nullptr;
  int32_t* expansions = nullptr;
  int64_t* done_ids = nullptr;                 // [G] game ids in the order they finished
  unsigned long long* done_count = nullptr;    // [1] (az_chess_selfplay_drain)
};

// MCTS.play through the tree API (az_chess_tree_play); all null/-1 in self-play
struct CPlayOut {
  const double* uniforms = nullptr;  // [slots] host random_sample draws; null: per-slot MT19937
  int greedy = -1;                   // -1: self_play.py:62's fullmove rule; 0/1: MCTS.play(greedy)
  int deterministic = 0;             // edge = argmax(probabilities) (mcts.py:199)
  int32_t* move = nullptr;           // [slots] move code, -1 idle
  int32_t* status = nullptr;         // [slots] outcome of the new root
  int32_t* pol_n = nullptr;          // [slots]
  int16_t* pol_a = nullptr;          // [slots][AZ_CHESS_MAX_MOVES]
  double* pol_p = nullptr;           // [slots][AZ_CHESS_MAX_MOVES]
};

constexpr int kMtN = 624;
constexpr int kStemFirstChunk = 2;  // input chunks of 32 planes the self-play stem skips

__device__ __forceinline__ Edge* arena(const CCfg& g, const CTree& t, int s, int h) {
  return t.edges + ((size_t)s * 2 + h) * g.half_cap;
}
__device__ __forceinline__ void flag(const CTree& t, unsigned long long f) {
  atomicOr(t.stats + az::kStatErrors, f);
}

// MT19937 per slot, word-major (az_tree.hip layout)
__device__ void mt_seed(const CTree& t, int s, uint32_t seed) {
  const int slots = t.mt_stride;
  uint32_t prev = seed;
  t.mt[s] = seed;
  for (int i = 1; i < kMtN; ++i) {
    prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
    t.mt[(size_t)i * slots + s] = prev;
  }
  t.mt[(size_t)kMtN * slots + s] = kMtN;
}
__device__ uint32_t mt_next(const CTree& t, int s) {
  const int slots = t.mt_stride;
  uint32_t* m = t.mt;
  uint32_t pos = m[(size_t)kMtN * slots + s];
  if (pos >= (uint32_t)kMtN) {
    for (int i = 0; i < kMtN; ++i) {
      const uint32_t y = (m[(size_t)i * slots + s] & 0x80000000u) |
                         (m[(size_t)((i + 1) % kMtN) * slots + s] & 0x7fffffffu);
      m[(size_t)i * slots + s] =
          m[(size_t)((i + 397) % kMtN) * slots + s] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    pos = 0;
  }
  const uint32_t y = m[(size_t)pos * slots + s];
  m[(size_t)kMtN * slots + s] = pos + 1;
  return az::mt_temper(y);
}
__device__ double mt_uniform(const CTree& t, int s) {
  const uint32_t a = mt_next(t, s) >> 5;
  const uint32_t b = mt_next(t, s) >> 6;
  return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

// numpy pairwise add.reduce (identity 0 + pairwise_sum, blocks of 128, 8
// accumulators) for n <= 256 (at most two levels of splitting)
template <typename T>
__device__ T pw_block(const T* a, int n) {
  if (n < 8) {
    T r = (T)0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  T r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}
template <typename T>
__device__ T pw_136(const T* a, int n) {
  if (n <= 128) return pw_block(a, n);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return pw_block(a, n2) + pw_block(a + n2, n - n2);
}
template <typename T>
__device__ T pairwise(const T* a, int n) {
  if (n <= 128) return pw_block(a, n);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return pw_136(a, n2) + pw_136(a + n2, n - n2);
}

// MCTS.backup (mcts.py:163-168): from the leaf's parent edge up, N + 1 and
// W + v with v negated per level -- by the slot's wave, one path level per
// lane (the levels are distinct edges): level d gets W + v * (-1)^(depth-1-d),
// the addend the serial walk gives it, so the same bits without the serial
// walk's chain of dependent loads (two memory round trips per level)
__device__ __forceinline__ void backup_wave(Edge* E, const int32_t* path, int depth, double v, int lane) {
  for (int d = lane; d < depth; d += 64) {
    Edge& e = E[path[d]];
    e.N += 1;
    e.W += ((depth - 1 - d) & 1) ? -v : v;
  }
}

__device__ void slot_reset(const CCfg& g, const CTree& t, const CSamples& smp, int s, int64_t gid) {
  az_chess_pos a;
  store_pos(start_pos(), a);
  t.root[s] = a;
  t.root_first[s] = 0;
  t.root_n[s] = 0;
  t.half[s] = 0;
  t.top[s] = 0;
  t.ply[s] = 0;
  t.initial[s] = 1;
  t.path_len[s] = 0;
  t.slot_exp[s] = 0;
  t.game_id[s] = gid;
  mt_seed(t, s, smp.base_seed + (uint32_t)gid);
}

// synthetic evaluator (oracle/chess_oracle.c orc_chess_synth): dyadic priors
// k/64 and values k/128 from a hash of the position the network would see
__device__ uint64_t pos_hash(const Pos& q, int initial) {
  uint64_t h = az::splitmix64(q.p[0]);
  for (int i = 1; i < 6; ++i) h = az::splitmix64(h ^ q.p[i]);
  h = az::splitmix64(h ^ q.co[0]);
  h = az::splitmix64(h ^ q.co[1]);
  h = az::splitmix64(h ^ q.castling);
  const uint64_t misc = (uint64_t)(uint16_t)q.ep | ((uint64_t)(uint16_t)q.half << 16) |
                        ((uint64_t)(uint16_t)q.full << 32) | ((uint64_t)initial << 48);
  return az::splitmix64(h ^ misc);
}

// ----------------------------------------------------------------- kernels

__global__ void slot_init_kernel(CCfg g, CTree t, CSamples smp, int64_t n_first) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.slots) return;
  if (s < n_first) slot_reset(g, t, smp, s, smp.first_game + s);
  else t.game_id[s] = -1;
}

// MCTS.__init__ (mcts.py:86-104) for the listed slots: a new root, no tree
__global__ void tree_reset_kernel(CCfg g, CTree t, int n, const int32_t* slots, const az_chess_pos* roots) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = slots[i];
  t.root[s] = roots[i];
  t.root_first[s] = 0;
  t.root_n[s] = 0;
  t.root_value[s] = 0.f;
  t.half[s] = 0;
  t.top[s] = 0;
  t.ply[s] = 0;
  t.initial[s] = 1;
  t.path_len[s] = 0;
  t.slot_exp[s] = 0;
  t.game_id[s] = s;
}

__global__ void tree_release_kernel(CTree t, int n, const int32_t* slots) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) t.game_id[slots[i]] = -1;
}

// ------------------------------------------------- transposition cache
// (az_tree.h's scheme: 16-slot buckets, LRU eviction by generations, a hit
// refreshes its entry into the current generation.)  The select wave that
// hits copies the payload into its slot's leaf_pay right away, so a reader
// holds an entry only for the few microseconds between its probe (which
// leaves the entry stamped with the current generation) and the copy: an
// insert evicts entries kCacheEvictAge+ generations old, and two generation
// turns (2 * cap / 16 inserts) cannot fall inside that window.
__device__ __forceinline__ uint64_t key_hash(const Pos& q, int initial) {
  return az::splitmix64(pos_hash(q, initial) ^ ((uint64_t)(uint32_t)q.turn << 8) ^ ((uint64_t)(uint32_t)q.rep << 16));
}
__device__ __forceinline__ uint32_t key_bucket(const ChessCache& c, uint64_t h) {
  return (uint32_t)h & c.mask & ~(uint32_t)(az::kCacheBucket - 1);
}
__device__ __forceinline__ bool same_key(const ChessKey* a, const az_chess_pos& pos, int initial) {
  const uint4* x = reinterpret_cast<const uint4*>(a);
  const uint4* y = reinterpret_cast<const uint4*>(&pos);
  uint4 v[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) v[i] = x[i];  // issued together: one round trip
  bool eq = v[5].x == (uint32_t)initial;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint4 w = y[i];
    eq = eq && v[i].x == w.x && v[i].y == w.y && v[i].z == w.z && v[i].w == w.w;
  }
  return eq;
}

// The wave's leaf (slot s, n legal moves) against the cache: true = a hit,
// its n priors and value copied to leaf_pay[s].  Lane 0 probes; every lane
// copies.
__device__ bool cache_probe_wave(const CTree& t, const ChessCache& c, int s, int lane, const az_chess_pos& key,
                                 int initial, uint64_t h, int n) {
  int idx = -1;
  if (lane == 0) {
    const uint32_t gen = (uint32_t)__hip_atomic_load(c.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t fp = az::cache_fp(h), base = key_bucket(c, h);
    uint32_t w[az::kCacheBucket];
#pragma unroll
    for (int k = 0; k < az::kCacheBucket; ++k)
      w[k] = __hip_atomic_load(c.state + base + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int hit = -1;
    uint32_t hst = 0;
    uint32_t cm = 0;  // fingerprint matches (buckets fill in slot order), then one acquire, then the keys
    bool stop = false;
#pragma unroll
    for (int k = 0; k < az::kCacheBucket; ++k) {
      const uint32_t st = w[k];
      if (stop) continue;
      if (st == az::kCacheEmpty) stop = true;
      else if ((st & 3u) == az::kCacheReady && (st >> 16) == fp) cm |= 1u << k;
    }
    if (cm) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      for (; cm; cm &= cm - 1) {
        const int k = __builtin_ctz(cm);
        if (same_key(c.keys + base + k, key, initial)) {
          hit = k;
#pragma unroll
          for (int kk = 0; kk < az::kCacheBucket; ++kk)
            if (kk == k) hst = w[kk];
          break;
        }
      }
    }
    if (hit >= 0 && az::cache_age(hst, gen) != 0) {
      // into the current generation (the LRU stamp); the CAS must win, or find
      // the entry moved there by another reader and still this key
      const uint32_t want = az::cache_word(fp, gen, az::kCacheReady);
      const uint32_t prev = atomicCAS(c.state + base + hit, hst, want);
      if (prev != hst) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (!(prev == want && same_key(c.keys + base + hit, key, initial))) hit = -1;
      }
    }
    idx = hit >= 0 ? (int)(base + hit) : -1;
  }
  idx = __shfl(idx, 0);
  if (idx < 0) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (every lane reads the payload)
  const float* src = c.pay + (size_t)idx * kPayFloats;
  float* dst = t.leaf_pay + (size_t)s * kPayFloats;
  for (int j = lane; j < n; j += 64) dst[j] = src[j];
  if (lane == 0) dst[AZ_CHESS_MAX_MOVES] = src[AZ_CHESS_MAX_MOVES];
  return true;
}

// plays_inferences[repr(board)] = (priors, value) (mcts.py:142) by the wave of
// the leaf's network row owner: the bucket's first empty slot, else its least
// recently used entry kCacheEvictAge+ generations old (az_tree.h); dropped
// when every entry is in use
__device__ void cache_insert_wave(const CTree& t, const ChessCache& c, int s, int lane, const float* sorted, int n,
                                  float value) {
  const az_chess_pos& key = t.leaf[s];
  const int initial = t.path_len[s] == 0 && t.initial[s];
  const Pos q = load_pos(key);
  const uint64_t h = key_hash(q, initial);
  int idx = -1;
  if (lane == 0) {
    const uint32_t gen = (uint32_t)__hip_atomic_load(c.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t fp = az::cache_fp(h), base = key_bucket(c, h);
    uint32_t w[az::kCacheBucket];
#pragma unroll
    for (int k = 0; k < az::kCacheBucket; ++k)
      w[k] = __hip_atomic_load(c.state + base + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t tried = 0;
    bool empty = false;
    for (int attempt = 0; attempt < az::kCacheBucket && idx < 0; ++attempt) {
      int pick = -1;
      uint32_t pst = 0, page = 0;
      bool pempty = false;
#pragma unroll
      for (int k = 0; k < az::kCacheBucket; ++k) {
        const uint32_t st = w[k];
        if (pempty || ((tried >> k) & 1u)) continue;
        if (st == az::kCacheEmpty) {
          pick = k, pst = st, pempty = true;
        } else if (c.gen_size) {
          const uint32_t age = az::cache_age(st, gen);
          if (age >= az::kCacheEvictAge && age > page) pick = k, pst = st, page = age;
        }
      }
      if (pick < 0) break;
      if (atomicCAS(c.state + base + pick, pst, az::cache_word(fp, gen, az::kCacheClaimed)) == pst) {
        idx = (int)(base + pick);
        empty = pempty;
      } else {
        tried |= 1u << pick;
      }
    }
    if (idx >= 0) {
      if (empty) atomicAdd(c.ctl + 2, 1ull);
      const unsigned long long m = atomicAdd(c.ctl + 1, 1ull) + 1;
      if (c.gen_size && m % c.gen_size == 0) atomicAdd(c.ctl, 1ull);
      atomicAdd(t.stats + az::kStatCacheInserts, 1ull);
    }
  }
  idx = __shfl(idx, 0);
  if (idx < 0) return;
  float* dst = c.pay + (size_t)idx * kPayFloats;
  for (int j = lane; j < n; j += 64) dst[j] = sorted[j];
  if (lane == 0) dst[AZ_CHESS_MAX_MOVES] = value;
  if (lane < 6) {
    uint4 v;
    if (lane < 5) v = reinterpret_cast<const uint4*>(&key)[lane];
    else v = make_uint4((uint32_t)initial, 0u, 0u, 0u);
    reinterpret_cast<uint4*>(c.keys + idx)[lane] = v;
  }
  // every lane's key and payload stores drained, then one agent release
  // before the publish (MI355X_MICROARCH.md, valid producer forms)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0)
    atomicExch(c.state + idx, az::cache_word(az::cache_fp(h),
                                             (uint32_t)__hip_atomic_load(c.ctl, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT),
                                             az::kCacheReady));
}

// MCTS.evaluate_and_expand (mcts.py:145-161) + backup of queue entry b
// (slot s) by one wave: the expand launch's, or -- fused -- the slot's wave
// in the next simulation's select launch, before its descent
struct ExpandSmem {
  int act[AZ_CHESS_MAX_MOVES];
  float sorted[AZ_CHESS_MAX_MOVES];
  float sum;
  int first_s;
};

// b: the slot's network row, or kQHit (its cached priors and value in leaf_pay).
// Round trips, each one's loads issued together: 1. the slot's counts, arena
// half and path (one level per lane), the leaf's value, first 64 moves and a
// hit's first 64 priors; 2. the path's edges and the moves' action indices;
// 3. the network row's priors -- where one load after another took eight.
__device__ void expand_body(const CCfg& g, const CTree& t, const ChessCache& c, const float* __restrict__ probs,
                            const float* __restrict__ values, int b, int s, int lane, ExpandSmem& sm) {
  int* act = sm.act;
  float* sorted = sm.sorted;
  const bool hit = b == kQHit;
  const int n = t.leaf_n[s];
  const int top = t.top[s];
  const int half = t.half[s];
  const int depth = t.path_len[s];
  const int32_t* path = t.path + (size_t)s * g.max_depth;
  const int pth = lane < g.max_depth ? path[lane] : 0;  // path level `lane` (past depth: stale, unused)
  const float* lp = t.leaf_pay + (size_t)s * kPayFloats;
  const float value = hit ? lp[AZ_CHESS_MAX_MOVES] : values[b];
  const int row_owner = hit ? -1 : t.eval_slot[b];
  const uint16_t* mv = t.leaf_moves + (size_t)s * AZ_CHESS_MAX_MOVES;
  const uint16_t m0 = mv[lane];  // moves 0..63 (64 < AZ_CHESS_MAX_MOVES)
  const float lp0 = hit ? lp[lane] : 0.f;
  Edge* E = arena(g, t, s, half);
  int en = 0;
  double ew = 0.0;
  if (lane < depth) {  // backup's loads now, its stores at the end (a path's edges are distinct)
    en = E[pth].N;
    ew = E[pth].W;
  }
  __syncthreads();
  if (hit) {  // plays_inferences[repr(board)] (mcts.py:123-128): the masked priors as stored
    for (int j = lane; j < n; j += 64) sorted[j] = j < 64 ? lp0 : lp[j];
  } else {
    const float* pr = probs + (size_t)b * AZ_CHESS_ACTIONS;
    for (int j = lane; j < n; j += 64) {
      const int a = action_of(t.lut, j < 64 ? m0 : mv[j]);
      act[j] = a;
      if (a < 0) flag(t, az::kErrIllegal);
    }
    __syncthreads();
    // probabilities[legal_moves_mask]: the legal actions in action order
    for (int j = lane; j < n; j += 64) {
      const int a = act[j];
      int r = 0;
      for (int i = 0; i < n; ++i) r += act[i] < a;
      sorted[r] = a >= 0 ? pr[a] : 0.f;
    }
  }
  __syncthreads();
  // the network row's owner publishes it (duplicates of this simulation share the row)
  const bool owner = !hit && row_owner == s;
  if (owner && c.enabled) cache_insert_wave(t, c, s, lane, sorted, n, value);
  if (lane == 0) {
    // normalize_probabilities (mcts/utils.py:4-16): the sum in numpy's
    // pairwise order here, the quotients per lane below
    sm.sum = pairwise(sorted, n);
    if (top + n > g.half_cap) {
      flag(t, az::kErrArena);
      sm.first_s = -1;
    } else {
      t.top[s] = top + n;
      sm.first_s = top;
    }
  }
  __syncthreads();
  const int first = sm.first_s;
  const float sum = sm.sum;
  if (first < 0) return;
  // zip(probabilities, node.board.moves): positional, python-chess move order
  for (int j = lane; j < n; j += 64) {
    Edge e;
    e.W = 0.0;
    e.prior = sum == 0.0f ? 1.0 / (double)n : (double)(float)(sorted[j] / sum);
    e.N = 0;
    e.child = az::kNoChild;
    e.child_n = 0;
    e.action = (int16_t)(j < 64 ? m0 : mv[j]);
    e.child_value = 0.f;
    E[first + j] = e;
  }
  const int leaf_edge = depth > 64 ? path[depth - 1] : __shfl(pth, depth > 0 ? depth - 1 : 0, 64);
  if (lane == 0) {
    if (depth == 0) {
      t.root_first[s] = first;
      t.root_n[s] = n;
      t.root_value[s] = value;
    } else {
      Edge& pe = E[leaf_edge];
      pe.child = first;
      pe.child_n = (int16_t)n;
      pe.child_value = value;
    }
  }
  // backup(-value) (mcts.py:175, 163-168): level d gets it negated depth - 1 - d times
  const double v = -(double)value;
  if (lane < depth) {
    E[pth].N = en + 1;
    E[pth].W = ew + (((depth - 1 - lane) & 1) ? -v : v);
  }
  for (int d = lane + 64; d < depth; d += 64) {  // levels past 64 (a long game's deep tree)
    Edge& e = E[path[d]];
    e.N += 1;
    e.W += ((depth - 1 - d) & 1) ? -v : v;
  }
  if (lane == 0) {
    t.slot_exp[s] += 1;
    atomicAdd(t.stats + az::kStatExpansions, 1ull);
    if (hit) atomicAdd(t.stats + az::kStatCacheHits, 1ull);
    else if (owner) atomicAdd(t.stats + az::kStatNNEvals, 1ull);
  }
}

// the leaf's is_game_over() (mcts.py:173-179): terminal leaves back up the
// canonical get_result (1 checkmate, 0 draw); others are queued for evaluation.
// One wave per slot: the wave generates the legal moves (legal_moves_wave,
// one square per lane; a single lane per slot took 19 us per launch), lane 0
// does the rest.
// (Round 5: run by the select launch's wave right after its descent, on the
// leaf in its registers -- one launch fewer on the lane's chain.)
// With the transposition cache on, an ongoing leaf is first looked up
// (cache_probe_wave: a hit copies its payload, slot_q = kQHit); a miss takes a
// network row unless an identical leaf of this simulation already did
// (per-simulation dedup: the step table's epoch-tagged fingerprint; a tag
// match is a candidate the launch's last block confirms by the full key).
__device__ __forceinline__ void leaf_body(const CCfg& g, const CTree& t, const ChessCache& c, int s, int lane,
                                          const Pos& q, uint16_t* cand) {
  bool check;
  const int n = legal_moves_wave(q, cand, t.leaf_moves + (size_t)s * AZ_CHESS_MAX_MOVES, &check, lane);
  if (n < 0) {  // wave-uniform
    if (lane == 0) {
      flag(t, az::kErrIllegal);
      t.slot_q[s] = -1;
    }
    return;
  }
  const int oc = outcome(q, n, check);  // wave-uniform
  if (oc != AZ_CHESS_ONGOING)
    backup_wave(arena(g, t, s, t.half[s]), t.path + (size_t)s * g.max_depth, t.path_len[s],
                oc == AZ_CHESS_CHECKMATE ? 1.0 : 0.0, lane);
  uint64_t h = 0;
  bool hit = false;
  if (oc == AZ_CHESS_ONGOING && c.enabled) {  // wave-uniform
    const int initial = t.path_len[s] == 0 && t.initial[s];
    h = key_hash(q, initial);
    az_chess_pos key;
    store_pos(q, key);
    hit = cache_probe_wave(t, c, s, lane, key, initial, h, n);
  }
  if (lane != 0) return;
  t.leaf_n[s] = n;
  int qi = -1;
  if (oc != AZ_CHESS_ONGOING) {
    atomicAdd(t.stats + az::kStatTerminal, 1ull);
  } else if (hit) {
    qi = kQHit;
  } else if (!c.enabled) {
    qi = atomicAdd(t.eval_count, 1);
    t.eval_slot[qi] = s;
  } else {
    const uint64_t tag = ((uint64_t)t.epoch << 32) | (uint32_t)(h >> 32);
    uint32_t sl = (uint32_t)h & t.step_mask;
    for (uint32_t p = 0; p <= t.step_mask; ++p) {
      const uint64_t cur = __hip_atomic_load(t.step_tag + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((uint32_t)(cur >> 32) != t.epoch) {  // empty in this epoch: try to own it
        const uint64_t prev = atomicCAS((unsigned long long*)(t.step_tag + sl), cur, tag);
        if (prev == cur) {
          qi = atomicAdd(t.eval_count, 1);
          t.eval_slot[qi] = s;
          t.step_row[sl] = qi;
          break;
        }
        if (prev != tag) continue;  // another tag took the slot: re-read it
      } else if (cur != tag) {
        sl = (sl + 1) & t.step_mask;
        continue;
      }
      qi = kQDup0 - (int)sl;  // a candidate duplicate: the last block confirms it
      t.dup_q[atomicAdd(t.dup_count, 1)] = s;
      break;
    }
  }
  t.slot_q[s] = qi;
  atomicAdd(t.stats + az::kStatSims, 1ull);
}

// The select launch's last block: its duplicate candidates get the owner's
// network row when the full keys (position + history form) agree, else a row
// of their own (a fingerprint collision).  Every block counts itself done
// after a device-scope fence; the block whose count completes the grid sees
// every block's queue stores.
__device__ void dup_tail(const CTree& t, const ChessCache& c, int lane) {
  if (!c.enabled) return;  // uniform
  __shared__ int last;
  // the wave's queue stores drained, one release, the count; the block that
  // completes it acquires (MI355X_MICROARCH.md, valid forms)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (lane == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = atomicAdd(t.sel_done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;  // block-uniform
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nd = __hip_atomic_load(t.dup_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int i = lane; i < nd; i += 64) {
    const int s2 = t.dup_q[i];
    const int sl = kQDup0 - t.slot_q[s2];
    const int row = t.step_row[sl];
    const int o = t.eval_slot[row];
    const int i2 = t.path_len[s2] == 0 && t.initial[s2], io = t.path_len[o] == 0 && t.initial[o];
    const uint4* a = reinterpret_cast<const uint4*>(t.leaf + s2);
    const uint4* b = reinterpret_cast<const uint4*>(t.leaf + o);
    bool same = i2 == io;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const uint4 x = a[k], y = b[k];
      same = same && x.x == y.x && x.y == y.y && x.z == y.z && x.w == y.w;
    }
    if (same) {
      t.slot_q[s2] = row;
    } else {
      const int r2 = atomicAdd(t.eval_count, 1);
      t.eval_slot[r2] = s2;
      t.slot_q[s2] = r2;
    }
  }
  __syncthreads();
  if (lane == 0) *t.sel_done = 0;  // the lane's next select launch counts from zero
}

// MCTS.select (mcts.py:111-120): one wave per slot, then the leaf's move
// generation and queueing (leaf_body).  FUSED: first the previous
// simulation's expand of the slot's queued leaf (expand_body; its network
// outputs are still in probs / values), so a search is select,
// (network, select) x (sims - 1), network, expand: one tree launch per
// simulation on the lane's chain instead of two
template <bool FUSED>
__device__ __forceinline__ void select_slot(const CCfg& g, const CTree& t, const ChessCache& c,
                                            const float* __restrict__ probs, const float* __restrict__ values,
                                            uint16_t* cand, ExpandSmem& esm) {
  const int s = blockIdx.x, lane = threadIdx.x;
  if (t.game_id[s] < 0) return;
  if constexpr (FUSED) {
    const int b = t.slot_q[s];  // wave-uniform
    if (b >= 0 || b == kQHit) {
      expand_body(g, t, c, probs, values, b, s, lane, esm);
      // the wave's edge and path stores complete before its descent reads them
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
  }
  const Edge* E = arena(g, t, s, t.half[s]);
  int32_t* path = t.path + (size_t)s * g.max_depth;
  Pos q = load_pos(t.root[s]);
  int first = t.root_first[s], cnt = t.root_n[s];
  int depth = 0;
  // below the root an expanded node's children's visits sum to its edge's
  // N - 1 (the first visit expanded it, every later one went on to a child),
  // so sqrt(sum) is read alongside the children's edges instead of after a
  // wave reduction over them: one dependent round trip per level, not two
  int sum_next = -1;
  while (cnt > 0) {
    int sum = sum_next;
    if (sum < 0) {  // the root: its children's visits, summed (wave-uniform)
      sum = 0;
      for (int j = lane; j < cnt; j += 64) sum += E[first + j].N;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    }
    if (sum >= g.pow_len) {
      if (lane == 0) flag(t, az::kErrPow);
      return;
    }
    const double sq = t.powtab[sum];
    double best_v = -INFINITY;
    int best = 1 << 30;
    for (int j = lane; j < cnt; j += 64) {
      const Edge e = E[first + j];
      const double qv = e.N ? e.W / (double)e.N : 0.0;
      const double u = g.c_puct * e.prior * sq / (double)(1 + e.N);
      const double v = qv + u;
      if (v > best_v) {  // within a lane j increases: strict > keeps the first
        best_v = v;
        best = j;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_xor(best_v, off, 64);
      const int oj = __shfl_xor(best, off, 64);
      if (ov > best_v || (ov == best_v && oj < best)) {  // np.argmax: first maximum
        best_v = ov;
        best = oj;
      }
    }
    if (depth >= g.max_depth) {
      if (lane == 0) flag(t, az::kErrPath);
      return;
    }
    const Edge e = E[first + best];
    if (lane == 0) path[depth] = first + best;
    ++depth;
    play(q, (uint16_t)e.action, true);  // Board.play(keep_same_player=True)
    first = e.child;
    cnt = e.child < 0 ? 0 : e.child_n;
    sum_next = e.N - 1;
  }
  if (lane == 0) {
    store_pos(q, t.leaf[s]);
    t.path_len[s] = depth;
  }
  leaf_body(g, t, c, s, lane, q, cand);
}
template <bool FUSED>
__global__ __launch_bounds__(64) void select_kernel(CCfg g, CTree t, ChessCache c, const float* __restrict__ probs,
                                                    const float* __restrict__ values) {
  __shared__ uint16_t cand[AZ_CHESS_MAX_MOVES];
  __shared__ ExpandSmem esm;
  // the next simulation's queue counters (this one's were zeroed by the last
  // simulation's launch; a memset launch per simulation cost 5 us)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *t.next_count = 0;
    if (t.next_dup) *t.next_dup = 0;
  }
  select_slot<FUSED>(g, t, c, probs, values, cand, esm);
  dup_tail(t, c, threadIdx.x);
}

// Board.full_state of the queued leaves into the network input [q][64][128]:
// history [0 x 6, start position, board] (every board made by play(), see
// chess/board.py docstring) or, for a root set by reset (the MCTS root is a
// deepcopy, whose copy() re-runs __init__), [0 x 7, start-position state]
// whatever the position -- the game's first Board() is the start position;
// the castling/counter planes are the board's own.  Planes 118..127 are the
// zero padding of the stem.  Written as split16 rows (AZ_CONV_F16X2; the
// plane values are small integers, exact in the first term) or fp32.
template <bool SPLIT>
__global__ __launch_bounds__(256) void encode_queue_kernel(CCfg g, CTree t, void* __restrict__ x) {
  __shared__ Pos sp[2];
  __shared__ float feat[6];
  __shared__ int initial;
  const int n = *t.eval_count;
  for (int b = blockIdx.x; b < n; b += gridDim.x) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const int s = t.eval_slot[b];
      sp[0] = start_pos();
      sp[1] = load_pos(t.leaf[s]);
      initial = t.path_len[s] == 0 && t.initial[s];
      float f[6];
      state_feats(sp[1], f);
      for (int i = 0; i < 6; ++i) feat[i] = f[i];
    }
    __syncthreads();
    const size_t row0 = (size_t)b * 64;
    float f[6];
    for (int i = 0; i < 6; ++i) f[i] = feat[i];
    for (int e2 = threadIdx.x; e2 < 64 * (32 - 8 * kStemFirstChunk); e2 += blockDim.x) {
      const int per = 32 - 8 * kStemFirstChunk;  // float4 per pixel written
      const int pix = e2 / per, e = pix * 32 + 8 * kStemFirstChunk + e2 % per;
      float v[4];
      full_state4(sp[0], sp[1], initial != 0, f, pix, (e & 31) * 4, v);
      az::store_act4<SPLIT>(x, row0 + pix, e & 31, make_float4(v[0], v[1], v[2], v[3]));
    }
  }
}

__global__ __launch_bounds__(256) void synth_kernel(CCfg g, CTree t, float* probs, float* values) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= *t.eval_count) return;
  const int s = t.eval_slot[b];
  const Pos q = load_pos(t.leaf[s]);
  const uint64_t h = pos_hash(q, t.path_len[s] == 0 && t.initial[s]);
  const uint64_t vh = az::splitmix64(h ^ 0x5555555555555555ull);
  values[b] = (float)(((double)(vh >> 56) - 128.0) / 128.0);
  float* p = probs + (size_t)b * AZ_CHESS_ACTIONS;
  if ((vh & 0x3F) == 0) {
    for (int a = 0; a < AZ_CHESS_ACTIONS; ++a) p[a] = 0.f;
    return;
  }
  uint64_t w = h;
  for (int a = 0; a < AZ_CHESS_ACTIONS; ++a) {
    if (a && a % 12 == 0) w = az::splitmix64(w);
    p[a] = (float)((double)(((w >> (5 * (a % 12))) & 31) + 1) / 64.0);
  }
}

// a search's last expand (its own launch): one wave per slot whose last
// simulation queued its leaf (a network row or a cache hit)
__global__ __launch_bounds__(64) void expand_kernel(CCfg g, CTree t, ChessCache c, const float* __restrict__ probs,
                                                    const float* __restrict__ values) {
  __shared__ ExpandSmem sm;
  const int s = blockIdx.x;
  if (t.game_id[s] < 0) return;
  const int b = t.slot_q[s];
  if (b >= 0 || b == kQHit) expand_body(g, t, c, probs, values, b, s, threadIdx.x, sm);
}

// MCTS.play (mcts.py:182-222) for every active slot + the self-play loop's
// bookkeeping (self_play.py:59-82); one wave per slot
__global__ __launch_bounds__(64) void play_kernel(CCfg g, CTree t, CSamples smp, CPlayOut po) {
  __shared__ double pi[AZ_CHESS_MAX_MOVES];
  __shared__ int chosen;
  __shared__ int done_code;
  const int s = blockIdx.x, lane = threadIdx.x;
  if (t.game_id[s] < 0) return;
  const int h = t.half[s];
  Edge* E = arena(g, t, s, h);
  Edge* D = arena(g, t, s, 1 - h);
  const int first = t.root_first[s], n = t.root_n[s];
  if (n <= 0) {
    if (lane == 0) flag(t, az::kErrNoRoot);
    return;
  }
  const bool tree_api = po.move != nullptr;
  const Pos root = load_pos(t.root[s]);
  const int64_t gid = t.game_id[s];
  const int64_t gi = gid - smp.first_game;
  const int ply = t.ply[s];
  for (int j = lane; j < n; j += 64) pi[j] = (double)E[first + j].N;
  __syncthreads();
  if (lane == 0) {
    const bool greedy = po.greedy < 0 ? root.full >= g.greedy_ply : po.greedy != 0;  // self_play.py:62
    if (greedy) {
      int im = 0;
      for (int i = 1; i < n; ++i)
        if (pi[i] > pi[im]) im = i;
      for (int i = 0; i < n; ++i) pi[i] = i == im ? 1.0 : 0.0;
    } else {
      const double sum = pairwise(pi, n);  // normalize_probabilities on float64 counts
      for (int i = 0; i < n; ++i) pi[i] = sum == 0.0 ? 1.0 / (double)n : pi[i] / sum;
    }
    if (po.deterministic) {
      int im = 0;  // np.argmax(probabilities): first maximum
      for (int i = 1; i < n; ++i)
        if (pi[i] > pi[im]) im = i;
      chosen = im;
    } else {
      // np.random.choice(edges, 1, p): one random_sample, cumsum, normalise, searchsorted right
      const double u = po.uniforms ? po.uniforms[s] : mt_uniform(t, s);
      double cdf[1];
      double acc = 0.0, last;
      for (int i = 0; i < n; ++i) acc += pi[i];
      last = acc;
      acc = 0.0;
      int idx = 0;
      for (int i = 0; i < n; ++i) {
        acc += pi[i];
        cdf[0] = acc / last;
        if (cdf[0] <= u) idx = i + 1;
      }
      chosen = idx < n ? idx : n - 1;
    }
  }
  __syncthreads();
  const int c_idx = chosen;
  const Edge c = E[first + c_idx];
  // sample record (MCTS.play return_details: parent state, policy, move)
  if (tree_api) {
    const size_t r = (size_t)s;
    for (int j = lane; j < n; j += 64) {
      po.pol_a[r * AZ_CHESS_MAX_MOVES + j] = (int16_t)action_of(t.lut, (uint16_t)E[first + j].action);
      po.pol_p[r * AZ_CHESS_MAX_MOVES + j] = pi[j];
    }
    if (lane == 0) {
      po.move[s] = (uint16_t)c.action;
      po.pol_n[s] = n;
    }
  } else if (gi >= 0 && gi < smp.n_games && ply < smp.plies) {
    const size_t r = (size_t)gi * smp.plies + ply;
    for (int j = lane; j < n; j += 64) {
      smp.pol_a[r * AZ_CHESS_MAX_MOVES + j] = (int16_t)action_of(t.lut, (uint16_t)E[first + j].action);
      smp.pol_p[r * AZ_CHESS_MAX_MOVES + j] = pi[j];
    }
    if (lane == 0) {
      smp.pos[r] = t.root[s];
      smp.moves[r] = (uint16_t)c.action;
      smp.pol_n[r] = n;
    }
  }
  // tree reuse: copy the chosen child's subtree into the other half
  // (Cheney scan: edges before `scan` point into D, edges after it into E)
  int top = 0;
  if (c.child >= 0) {
    for (int j = lane; j < c.child_n; j += 64) D[j] = E[c.child + j];
    top = c.child_n;
  }
  __syncthreads();
  int scan = 0;
  bool overflow = false;
  while (scan < top) {
    const int top0 = top;
    const int j = scan + lane;
    Edge e;
    int need = 0;
    if (j < top0) {
      e = D[j];
      if (e.child >= 0) need = e.child_n;
    }
    int incl = need;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    const int total = __shfl(incl, 63, 64);
    if (top0 + total > g.half_cap) {
      overflow = true;
      break;
    }
    if (need) {
      const int nf = top0 + incl - need;
      for (int k = 0; k < need; ++k) D[nf + k] = E[e.child + k];
      e.child = nf;
      D[j] = e;
    }
    top = top0 + total;
    scan = min(scan + 64, top0);
    __syncthreads();
  }
  if (lane == 0) {
    if (overflow) flag(t, az::kErrArena);
    Pos nr = root;
    play(nr, (uint16_t)c.action, true);
    az_chess_pos a;
    store_pos(nr, a);
    t.root[s] = a;
    t.half[s] = 1 - h;
    t.top[s] = overflow ? 0 : top;
    t.root_first[s] = 0;
    t.root_n[s] = (c.child >= 0 && !overflow) ? c.child_n : 0;
    t.ply[s] = ply + 1;
    t.initial[s] = 0;
    atomicAdd(t.stats + az::kStatPlies, 1ull);
    // while not mcts.board.is_game_over() (self_play.py:59)
    bool check;
    const int nl = legal_moves(nr, t.leaf_moves + (size_t)s * AZ_CHESS_MAX_MOVES, &check);
    int oc = nl < 0 ? AZ_CHESS_ONGOING : outcome(nr, nl, check);
    if (tree_api) {
      po.status[s] = oc;  // the MCTS object keeps its (possibly finished) board
      oc = AZ_CHESS_ONGOING;
    } else if (oc == AZ_CHESS_ONGOING && ply + 1 >= g.max_plies) {
      oc = AZ_CHESS_MAX_PLIES;
    }
    done_code = oc;
  }
  __syncthreads();
  if (done_code != AZ_CHESS_ONGOING && lane == 0) {
    if (gi >= 0 && gi < smp.n_games) {
      smp.length[gi] = ply + 1;
      smp.result[gi] = done_code == AZ_CHESS_CHECKMATE ? 1 : 0;
      smp.term[gi] = done_code;
      smp.expansions[gi] = t.slot_exp[s];
      // the drain's finish-order list (its records are complete: stored above)
      if (smp.done_ids) {
        __threadfence();
        smp.done_ids[atomicAdd(smp.done_count, 1ull)] = smp.first_game + gi;
      }
    }
    atomicAdd(t.stats + az::kStatGamesDone, 1ull);
    const unsigned long long next = atomicAdd(t.stats + az::kStatNextGame, 1ull);
    if ((int64_t)next < smp.first_game + smp.n_games) slot_reset(g, t, smp, s, (int64_t)next);
    else t.game_id[s] = -1;
  }
}

#define AZC_HIP(expr)                                                                      \
  do {                                                                                     \
    hipError_t err__ = (expr);                                                             \
    if (err__ != hipSuccess)                                                               \
      return az::fail_abi(AZ_E_HIP, std::string(#expr) + ": " + hipGetErrorString(err__)); \
  } while (0)

}  // namespace
}  // namespace azc

using namespace azc;

// A lane = a contiguous slot group searched on its own HIP stream: its
// simulations' tree kernels and network launches overlap the other lanes'
// (a 256-game step is latency-bound: one launch fills half the CUs).
struct CLane {
  int first = 0;
  hipStream_t stream = nullptr;
  CCfg g{};
  CTree t{};
  float* x = nullptr;
  float* act[3] = {nullptr, nullptr, nullptr};
  float* probs = nullptr;
  float* values = nullptr;
  az::ConvTimer timer;
  int32_t* counts = nullptr;  // [2] the eval queue counters, alternating by simulation
  int par = 0;
  bool pending_expand = false;  // the last simulation's expand not launched yet
  hipEvent_t move_done[4] = {nullptr, nullptr, nullptr, nullptr};  // move m's end on this lane (m % 4)
  ChessCache cache{};  // the engine's (flush_expand has no engine pointer)
};

struct az_chess_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  az_chess_config cfg{};
  CCfg g{};
  CTree t{};
  std::vector<CLane*> lanes;
  CSamples smp{};
  ChessCache cache{};  // the transposition cache (az_chess_config.cache_log2; enabled = 0 when off)
  az::NetDev net{};
  az::ConvTimer timer;
  hipEvent_t timer_ref = nullptr;
  float* x = nullptr;
  float* act[3] = {nullptr, nullptr, nullptr};
  float* probs = nullptr;
  float* values = nullptr;
  std::vector<void*> owned, sample_bufs;
  int64_t sp_n = 0;
  // asynchronous steps + drain (ABI 10), as the Connect-N engine: per move m
  // the last lane to finish it stores the games-finished count into pinned
  // snap_host[m % 4] (az::launch_move_end); the drain copies the games of the
  // newest move whose snapshot is complete on pack_stream
  int64_t moves_issued = 0, batch_first_move = 0, drained = 0;
  int32_t* move_arrive = nullptr;           // device [4]
  unsigned long long* snap_dev = nullptr;   // pinned [4] (device view)
  unsigned long long* snap_host = nullptr;  // its host view
  hipStream_t pack_stream = nullptr;
  // tree API staging (allocated on first use)
  double* tree_u = nullptr;
  int32_t *tree_move = nullptr, *tree_status = nullptr, *tree_pol_n = nullptr, *tree_slots = nullptr;
  int16_t* tree_pol_a = nullptr;
  double* tree_pol_p = nullptr;
  az_chess_pos* tree_roots = nullptr;

  template <typename T>
  int alloc(T** p, size_t count) {
    void* q = nullptr;
    AZC_HIP(hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)));
    owned.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return 0;
  }
};

namespace {

int check_errors(az_chess_engine* e) {
  unsigned long long err = 0;
  AZC_HIP(hipMemcpy(&err, e->t.stats + az::kStatErrors, sizeof(err), hipMemcpyDeviceToHost));
  if (!err) return 0;
  std::string m = "device error flags:";
  if (err & az::kErrArena) m += " arena-overflow(raise az_chess_config.arena_edges)";
  if (err & az::kErrPow) m += " visit-table-overflow";
  if (err & az::kErrPath) m += " path-overflow";
  if (err & az::kErrIllegal) m += " illegal-move";
  if (err & az::kErrNoRoot) m += " play-before-search";
  if (err & az::kErrActRange)
    m += " activation-range(a non-finite activation, or |x| > 32752 in the per-layer fp16x2 convs: "
         "use conv_algo=AZ_CONV_F16X2 or AZ_CONV_DIRECT)";
  // play on a slot without a searched root changes nothing: that flag is
  // cleared once reported (the others mean a broken tree and stay)
  if (err == az::kErrNoRoot) AZC_HIP(hipMemset(e->t.stats + az::kStatErrors, 0, sizeof(err)));
  return az::fail_abi(AZ_E_DEVICE, m);
}

int simulate(az_chess_engine* e, CLane& L) {
  hipStream_t s = L.stream;
  const int S = L.g.slots;
  // the queue and duplicate counters: one pair per simulation parity (the
  // select launch zeroes the other pair, the next simulation's)
  L.t.eval_count = L.counts + 2 * L.par;
  L.t.dup_count = L.counts + 2 * L.par + 1;
  L.t.next_count = L.counts + 2 * (L.par ^ 1);
  L.t.next_dup = L.counts + 2 * (L.par ^ 1) + 1;
  L.par ^= 1;
  L.t.epoch += 1;  // a fresh dedup table (tags of older epochs read as empty)
  if (L.pending_expand) select_kernel<true><<<S, 64, 0, s>>>(L.g, L.t, e->cache, L.probs, L.values);
  else select_kernel<false><<<S, 64, 0, s>>>(L.g, L.t, e->cache, nullptr, nullptr);
  if (L.g.evaluator == AZ_EVAL_NETWORK) {
    // the one-launch tower builds the leaves' input planes itself (no encode
    // launch on the chain; az_nn.h TowerLeaves); the other forms read rows
    const bool tower = e->net.algo == AZ_CONV_F16X2 && e->net.use_tower && e->net.tower;
    az::TowerLeaves lv;
    lv.eval_slot = L.t.eval_slot;
    lv.leaf = L.t.leaf;
    lv.path_len = L.t.path_len;
    lv.initial = L.t.initial;
    if (!tower) {
      if (e->net.algo == AZ_CONV_F16X2)
        encode_queue_kernel<true><<<std::min(S, 2048), 256, 0, s>>>(L.g, L.t, L.x);
      else
        encode_queue_kernel<false><<<std::min(S, 2048), 256, 0, s>>>(L.g, L.t, L.x);
    }
    // history slots 0-5 (planes 0-83) are always empty in self-play (every
    // board's history is [0 x 6, start, board] or [0 x 7, start]): the stem
    // skips input chunks 0-1 (planes 0-63; they would add exact zeros) and
    // the planes 64-127 only are written
    az::launch_forward(e->net, L.x, L.t.eval_count, S, 8, 8, AZ_CHESS_ACTIONS, L.act[0], L.act[1],
                       L.act[2], L.probs, L.values, s, L.timer.enabled ? &L.timer : nullptr, nullptr,
                       kStemFirstChunk, tower ? &lv : nullptr);
  } else {
    synth_kernel<<<(S + 255) / 256, 256, 0, s>>>(L.g, L.t, L.probs, L.values);
  }
  L.pending_expand = true;  // in the next simulation's select launch, or flush_expand
  AZC_HIP(hipGetLastError());
  return 0;
}

// the last simulation's expand of a search (its own launch, by queue entry)
int flush_expand(CLane& L) {
  if (!L.pending_expand) return 0;
  L.pending_expand = false;
  expand_kernel<<<L.g.slots, 64, 0, L.stream>>>(L.g, L.t, L.cache, L.probs, L.values);
  AZC_HIP(hipGetLastError());
  return 0;
}

int sync_lanes(az_chess_engine* e) {
  for (CLane* L : e->lanes) AZC_HIP(hipStreamSynchronize(L->stream));
  AZC_HIP(hipStreamSynchronize(e->stream));
  return 0;
}

// lane view: per-slot arrays offset to the lane's first slot, its own eval
// queue counter and evaluator buffer slices
int make_lane(az_chess_engine* e, CLane* L, int first, int n) {
  L->first = first;
  L->g = e->g;
  L->g.slots = n;
  CTree t = e->t;
  const size_t f = (size_t)first;
  t.edges += f * 2 * e->g.half_cap;
  t.root += f;
  t.root_first += f;
  t.root_n += f;
  t.half += f;
  t.top += f;
  t.ply += f;
  t.initial += f;
  t.game_id += f;
  t.path += f * e->g.max_depth;
  t.path_len += f;
  t.leaf += f;
  t.leaf_moves += f * AZ_CHESS_MAX_MOVES;
  t.leaf_n += f;
  t.slot_exp += f;
  t.root_value += f;
  t.mt += f;
  t.eval_slot += f;
  t.slot_q += f;
  if (t.leaf_pay) t.leaf_pay += f * kPayFloats;
  int rc;
  if ((rc = e->alloc(&t.eval_count, 4))) return rc;
  AZC_HIP(hipMemset(t.eval_count, 0, 4 * sizeof(int32_t)));
  L->counts = t.eval_count;
  t.dup_count = t.eval_count + 1;
  t.next_count = t.eval_count + 2;
  t.next_dup = t.eval_count + 3;
  // the lane's per-simulation dedup table (load factor <= 25%) and duplicates list
  size_t cap = 256;
  while (cap < 4 * (size_t)n) cap <<= 1;
  if ((rc = e->alloc(&t.step_tag, cap)) || (rc = e->alloc(&t.step_row, cap)) || (rc = e->alloc(&t.dup_q, n)) ||
      (rc = e->alloc(&t.sel_done, 1)))
    return rc;
  AZC_HIP(hipMemset(t.step_tag, 0, cap * sizeof(uint64_t)));
  AZC_HIP(hipMemset(t.sel_done, 0, sizeof(uint32_t)));
  t.step_mask = (uint32_t)(cap - 1);
  t.epoch = 0;
  L->cache = e->cache;
  L->t = t;
  if (e->x) L->x = e->x + f * 64 * 128;
  for (int i = 0; i < 3; ++i) L->act[i] = e->act[i] ? e->act[i] + f * 64 * 128 : nullptr;
  L->probs = e->probs + f * AZ_CHESS_ACTIONS;
  L->values = e->values + f;
  if (hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking) != hipSuccess)
    return az::fail_abi(AZ_E_HIP, "hipStreamCreate failed");
  return 0;
}

}  // namespace

extern "C" {

int az_chess_engine_create(int device, const az_chess_config* cfg, az_chess_engine** out) {
  if (!cfg || !out) return az::fail_abi(AZ_E_INVALID, "null argument");
  const az_chess_config& c = *cfg;
  if (c.slots < 1 || c.mcts_iterations < 1) return az::fail_abi(AZ_E_INVALID, "slots and mcts_iterations must be >= 1");
  if (c.evaluator != AZ_EVAL_NETWORK && c.evaluator != AZ_EVAL_SYNTHETIC)
    return az::fail_abi(AZ_E_INVALID, "unknown evaluator");
  if (c.evaluator == AZ_EVAL_NETWORK && c.filters != 128)
    return az::fail_abi(AZ_E_INVALID, "network evaluator supports filters == 128 (ConfigModel.filters)");
  if (c.conv_algo != AZ_CONV_F16X2 && c.conv_algo != AZ_CONV_DIRECT && c.conv_algo != AZ_CONV_F16X2_LAYERS)
    return az::fail_abi(AZ_E_INVALID, "conv_algo must be AZ_CONV_F16X2, AZ_CONV_DIRECT or AZ_CONV_F16X2_LAYERS");
  if (c.max_plies < 0 || c.arena_edges < 0 || c.depth < 0 || c.value_hidden < 1)
    return az::fail_abi(AZ_E_INVALID, "negative bound");
  if ((int64_t)c.slots * 64 * 512 >= (1ll << 31))
    return az::fail_abi(AZ_E_INVALID, "slots * 64 * 512 must stay below 2^31 (32-bit activation byte offsets)");
  int dev_count = 0;
  if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count == 0)
    return az::fail_abi(AZ_E_HIP, "no HIP device visible: libaz has no CPU fallback");
  if (device < 0 || device >= dev_count) return az::fail_abi(AZ_E_INVALID, "bad device index");
  AZC_HIP(hipSetDevice(device));
  AZC_HIP(upload_rays());
  az_chess_engine* e = new az_chess_engine();
  e->device = device;
  e->cfg = c;
  CCfg& g = e->g;
  g.slots = c.slots;
  g.sims = c.mcts_iterations;
  g.greedy_ply = c.index_move_greedy;
  g.c_puct = c.exploration_constant;
  g.evaluator = c.evaluator;
  g.max_plies = c.max_plies > 0 ? c.max_plies : 512;
  g.max_depth = 512;
  const int64_t half = c.arena_edges > 0 ? c.arena_edges : (int64_t)96 * c.mcts_iterations + 256;
  const int64_t visits = (int64_t)c.mcts_iterations * g.max_plies + 2;
  if (half > (1 << 30) || visits > (1 << 28) || (int64_t)c.slots * 2 * half > (1ll << 36)) {
    delete e;
    return az::fail_abi(AZ_E_INVALID, "tree bounds too large");
  }
  g.half_cap = (int)half;
  g.pow_len = (int)visits;
  auto cleanup = [&](int rc) {
    az_chess_engine_destroy(e);
    return rc;
  };
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(az::fail_abi(AZ_E_HIP, "hipStreamCreate failed"));
  const size_t S = (size_t)g.slots;
  CTree& t = e->t;
  int rc;
  if ((rc = e->alloc(&t.edges, S * 2 * (size_t)g.half_cap)) || (rc = e->alloc(&t.root, S)) ||
      (rc = e->alloc(&t.root_first, S)) || (rc = e->alloc(&t.root_n, S)) || (rc = e->alloc(&t.half, S)) ||
      (rc = e->alloc(&t.top, S)) || (rc = e->alloc(&t.ply, S)) || (rc = e->alloc(&t.initial, S)) ||
      (rc = e->alloc(&t.game_id, S)) || (rc = e->alloc(&t.path, S * g.max_depth)) ||
      (rc = e->alloc(&t.path_len, S)) || (rc = e->alloc(&t.leaf, S)) ||
      (rc = e->alloc(&t.leaf_moves, S * AZ_CHESS_MAX_MOVES)) || (rc = e->alloc(&t.leaf_n, S)) ||
      (rc = e->alloc(&t.slot_exp, S)) || (rc = e->alloc(&t.root_value, S)) ||
      (rc = e->alloc(&t.mt, S * (kMtN + 1))) ||
      (rc = e->alloc(&t.eval_slot, S)) || (rc = e->alloc(&t.eval_count, 1)) || (rc = e->alloc(&t.slot_q, S)) ||
      (rc = e->alloc(&t.stats, az::kStatCount)))
    return cleanup(rc);
  t.next_count = t.eval_count;  // (the lanes' views carry their own pair)
  {
    double* powtab = nullptr;
    if ((rc = e->alloc(&powtab, g.pow_len))) return cleanup(rc);
    std::vector<double> hp(g.pow_len);
    double (*volatile pw)(double, double) = pow;  // libm pow, as Python `** 0.5` (mcts.py:50)
    for (int k = 0; k < g.pow_len; ++k) hp[k] = k == 0 ? 0.0 : pw((double)k, 0.5);
    if (hipMemcpy(powtab, hp.data(), hp.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(az::fail_abi(AZ_E_HIP, "pow table upload failed"));
    t.powtab = powtab;
    int16_t* lut = nullptr;
    std::vector<int16_t> hl = action_lut();
    if ((rc = e->alloc(&lut, hl.size()))) return cleanup(rc);
    if (hipMemcpy(lut, hl.data(), hl.size() * sizeof(int16_t), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(az::fail_abi(AZ_E_HIP, "action table upload failed"));
    t.lut = lut;
  }
  if (hipMemset(t.stats, 0, az::kStatCount * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(t.game_id, 0xff, S * sizeof(int64_t)) != hipSuccess)
    return cleanup(az::fail_abi(AZ_E_HIP, "memset failed"));
  if ((rc = e->alloc(&e->probs, S * AZ_CHESS_ACTIONS)) || (rc = e->alloc(&e->values, S))) return cleanup(rc);
  if (c.evaluator == AZ_EVAL_NETWORK) {
    if ((rc = e->alloc(&e->x, S * 64 * 128))) return cleanup(rc);
    if (hipMemset(e->x, 0, S * 64 * 128 * sizeof(float)) != hipSuccess)
      return cleanup(az::fail_abi(AZ_E_HIP, "memset failed"));
    for (int i = 0; i < 3; ++i)
      if ((rc = e->alloc(&e->act[i], S * 64 * 128))) return cleanup(rc);
  }
  t.mt_stride = g.slots;
  // the transposition cache (mcts.py:122-143 on chess boards)
  if (c.cache_log2 < 0 || c.cache_log2 > 28 || (c.cache_log2 > 0 && c.cache_log2 < 4))
    return cleanup(az::fail_abi(AZ_E_INVALID, "cache_log2 must be 0 (no cache) or 4..28"));
  t.leaf_pay = nullptr;
  if (c.cache_log2 > 0) {
    const size_t cap = (size_t)1 << c.cache_log2;
    ChessCache& cc = e->cache;
    if ((rc = e->alloc(&cc.keys, cap)) || (rc = e->alloc(&cc.state, cap)) ||
        (rc = e->alloc(&cc.pay, cap * kPayFloats)) || (rc = e->alloc(&cc.ctl, 4)) ||
        (rc = e->alloc(&t.leaf_pay, S * kPayFloats)))
      return cleanup(rc);
    cc.mask = (uint32_t)(cap - 1);
    cc.enabled = 1;
    // LRU by generations of cap/16 inserts (a reader holds an entry only
    // between its probe and its payload copy, inside one select launch)
    cc.gen_size = cap / az::kCacheGenDiv;
    if (hipMemset(cc.state, 0, cap * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(cc.ctl, 0, 4 * sizeof(unsigned long long)) != hipSuccess)
      return cleanup(az::fail_abi(AZ_E_HIP, "cache memset failed"));
  }
  e->net.depth = c.depth;
  // depth 0: the fp16x2 chain runs the heads' 1x1 convs inside the last
  // block's conv2, so a tower without blocks takes the fp32 MFMA path
  e->net.algo = c.depth == 0 ? AZ_CONV_DIRECT : (c.conv_algo == AZ_CONV_F16X2_LAYERS ? AZ_CONV_F16X2 : c.conv_algo);
  // AZ_CONV_F16X2: the stem, the tower and the heads' 1x1 convs in one launch
  // (tower16_kernel's input-row form) when the network fits it, else the
  // per-layer conv16 chain (AZ_CONV_F16X2_LAYERS forces the chain)
  e->net.use_tower = c.conv_algo == AZ_CONV_F16X2 && c.depth >= 1 && c.depth <= az::kTowerMaxDepth;
  e->net.board_h = e->net.board_w = 8;
  e->net.hidden = c.value_hidden;
  e->net.err = t.stats + az::kStatErrors;
  if (c.lanes < 0) return cleanup(az::fail_abi(AZ_E_INVALID, "lanes must be >= 0"));
  // auto = 2 from 128 games: a lane's simulation is a latency-bound chain of
  // ~14 launches, and a second stream's chain fills the CUs its small kernels
  // leave idle (round 2, conv16: 1 lane 1.17M expansions/s, 2 lanes 1.37-1.42M,
  // 3-4 lanes 0.82M -- tiny per-lane batches, and the streams then share
  // the 4 hardware queues; profiles/r2/chess_lanes.txt)
  int nl = c.lanes > 0 ? c.lanes : (g.slots >= 128 ? 2 : 1);
  nl = std::min(nl, std::min(g.slots, 16));
  for (int l = 0; l < nl; ++l) {
    CLane* L = new CLane();
    e->lanes.push_back(L);
    const int lo = (int)((int64_t)g.slots * l / nl), hi = (int)((int64_t)g.slots * (l + 1) / nl);
    if ((rc = make_lane(e, L, lo, hi - lo))) return cleanup(rc);
    for (hipEvent_t& ev : L->move_done)
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
        return cleanup(az::fail_abi(AZ_E_HIP, "hipEventCreate failed"));
  }
  // the drain's move snapshots (pinned, coherent) and its own stream
  if ((rc = e->alloc(&e->move_arrive, 4))) return cleanup(rc);
  if (hipMemset(e->move_arrive, 0, 4 * sizeof(int32_t)) != hipSuccess ||
      hipHostMalloc(&e->snap_host, 4 * sizeof(unsigned long long), hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&e->snap_dev, e->snap_host, 0) != hipSuccess ||
      hipStreamCreateWithFlags(&e->pack_stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(az::fail_abi(AZ_E_HIP, "drain snapshot allocation failed"));
  for (int i = 0; i < 4; ++i) e->snap_host[i] = 0;
  *out = e;
  return 0;
}

int az_chess_engine_destroy(az_chess_engine* e) {
  if (!e) return 0;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (CLane* L : e->lanes) {
    if (L->stream) {
      (void)hipStreamSynchronize(L->stream);
      (void)hipStreamDestroy(L->stream);
    }
    for (hipEvent_t ev : L->move_done)
      if (ev) (void)hipEventDestroy(ev);
    delete L;
  }
  if (e->pack_stream) {
    (void)hipStreamSynchronize(e->pack_stream);
    (void)hipStreamDestroy(e->pack_stream);
  }
  if (e->snap_host) (void)hipHostFree(e->snap_host);
  for (void* p : e->sample_bufs) (void)hipFree(p);
  for (void* p : e->owned) (void)hipFree(p);
  if (e->timer_ref) (void)hipEventDestroy(e->timer_ref);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return 0;
}

int az_chess_engine_set_weights(az_chess_engine* e, const az_tensor* tensors, int n) {
  if (!e || (!tensors && n)) return az::fail_abi(AZ_E_INVALID, "null argument");
  if (e->cfg.evaluator != AZ_EVAL_NETWORK) return az::fail_abi(AZ_E_STATE, "engine has no network evaluator");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  if ((rc = sync_lanes(e))) return rc;
  if (e->cache.state) {  // a new model empties plays_inferences (self_play.py:145-146)
    AZC_HIP(hipMemset(e->cache.state, 0, ((size_t)e->cache.mask + 1) * sizeof(uint32_t)));
    AZC_HIP(hipMemset(e->cache.ctl, 0, 4 * sizeof(unsigned long long)));
  }
  return az::load_network(e->net, tensors, n, AZ_CHESS_PLANES, 64, AZ_CHESS_ACTIONS, e->cfg.bn_epsilon,
                          e->owned);
}

int az_chess_forward(az_chess_engine* e, const float* x, int n, float* probs, float* values) {
  if (!e || n < 0 || (n && (!x || !probs || !values))) return az::fail_abi(AZ_E_INVALID, "bad arguments");
  if (!e->net.ready) return az::fail_abi(AZ_E_STATE, "az_chess_engine_set_weights was not called");
  AZC_HIP(hipSetDevice(e->device));
  const int chunk = e->g.slots;
  for (int off = 0; off < n; off += chunk) {
    const int m = std::min(chunk, n - off);
    // [m][64][118] -> the network input [m][64][128] (planes 118..127 zero), split16 for the
    // fp16x2 convs; act[2] stages the host floats (the forward writes it only after the stem)
    float* staging = static_cast<float*>(e->act[2]);
    AZC_HIP(hipMemcpyAsync(staging, x + (size_t)off * 64 * AZ_CHESS_PLANES,
                           (size_t)m * 64 * AZ_CHESS_PLANES * sizeof(float), hipMemcpyHostToDevice, e->stream));
    az::launch_pad_rows(staging, m * 64, AZ_CHESS_PLANES, e->x, e->net.algo == AZ_CONV_F16X2, e->stream);
    az::launch_forward(e->net, e->x, nullptr, m, 8, 8, AZ_CHESS_ACTIONS, e->act[0], e->act[1], e->act[2],
                       e->probs, e->values, e->stream, e->timer.enabled ? &e->timer : nullptr);
    AZC_HIP(hipGetLastError());
    AZC_HIP(hipMemcpyAsync(probs + (size_t)off * AZ_CHESS_ACTIONS, e->probs,
                           (size_t)m * AZ_CHESS_ACTIONS * sizeof(float), hipMemcpyDeviceToHost, e->stream));
    AZC_HIP(hipMemcpyAsync(values + off, e->values, (size_t)m * sizeof(float), hipMemcpyDeviceToHost, e->stream));
    AZC_HIP(hipStreamSynchronize(e->stream));
  }
  return 0;
}

int az_chess_selfplay_begin(az_chess_engine* e, int64_t first_game, int64_t n_games, uint32_t base_seed) {
  if (!e || n_games < 0 || first_game < 0) return az::fail_abi(AZ_E_INVALID, "bad arguments");
  if (e->cfg.evaluator == AZ_EVAL_NETWORK && !e->net.ready)
    return az::fail_abi(AZ_E_STATE, "network evaluator selected but az_chess_engine_set_weights was not called");
  AZC_HIP(hipSetDevice(e->device));
  for (CLane* L : e->lanes) L->pending_expand = false;  // (a search an error interrupted)
  int rc;
  if ((rc = sync_lanes(e))) return rc;
  for (void* p : e->sample_bufs) (void)hipFree(p);
  e->sample_bufs.clear();
  CSamples& smp = e->smp;
  smp = CSamples{};
  smp.first_game = first_game;
  smp.n_games = n_games;
  smp.base_seed = base_seed;
  smp.plies = e->g.max_plies;
  const size_t G = (size_t)std::max<int64_t>(n_games, 1), P = (size_t)smp.plies, M = AZ_CHESS_MAX_MOVES;
  auto get = [&](void** p, size_t bytes) -> int {
    AZC_HIP(hipMalloc(p, std::max<size_t>(bytes, 16)));
    e->sample_bufs.push_back(*p);
    AZC_HIP(hipMemsetAsync(*p, 0, std::max<size_t>(bytes, 16), e->stream));
    return 0;
  };
  if ((rc = get((void**)&smp.pos, G * P * sizeof(az_chess_pos))) ||
      (rc = get((void**)&smp.moves, G * P * sizeof(uint16_t))) ||
      (rc = get((void**)&smp.pol_n, G * P * sizeof(int32_t))) ||
      (rc = get((void**)&smp.pol_a, G * P * M * sizeof(int16_t))) ||
      (rc = get((void**)&smp.pol_p, G * P * M * sizeof(double))) ||
      (rc = get((void**)&smp.length, G * sizeof(int32_t))) || (rc = get((void**)&smp.result, G * sizeof(int32_t))) ||
      (rc = get((void**)&smp.term, G * sizeof(int32_t))) || (rc = get((void**)&smp.expansions, G * sizeof(int32_t))) ||
      (rc = get((void**)&smp.done_ids, G * sizeof(int64_t))) ||
      (rc = get((void**)&smp.done_count, sizeof(unsigned long long))))
    return rc;
  e->drained = 0;
  e->batch_first_move = e->moves_issued;
  unsigned long long st[az::kStatCount] = {0};
  const int64_t first_wave = std::min<int64_t>(n_games, e->g.slots);
  st[az::kStatNextGame] = (unsigned long long)(first_game + first_wave);
  AZC_HIP(hipMemcpyAsync(e->t.stats, st, sizeof(st), hipMemcpyHostToDevice, e->stream));
  slot_init_kernel<<<(e->g.slots + 255) / 256, 256, 0, e->stream>>>(e->g, e->t, smp, first_wave);
  AZC_HIP(hipGetLastError());
  AZC_HIP(hipStreamSynchronize(e->stream));
  e->sp_n = n_games;
  return 0;
}

int az_chess_stats(az_chess_engine* e, az_stats* st) {
  if (!e || !st) return az::fail_abi(AZ_E_INVALID, "null argument");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  if ((rc = sync_lanes(e))) return rc;
  unsigned long long h[az::kStatCount];
  AZC_HIP(hipMemcpy(h, e->t.stats, sizeof(h), hipMemcpyDeviceToHost));
  std::vector<int64_t> gid(e->g.slots);
  AZC_HIP(hipMemcpy(gid.data(), e->t.game_id, gid.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
  memset(st, 0, sizeof(*st));
  st->expansions = (int64_t)h[az::kStatExpansions];
  st->terminal_visits = (int64_t)h[az::kStatTerminal];
  st->games_done = (int64_t)h[az::kStatGamesDone];
  st->simulations = (int64_t)h[az::kStatSims];
  st->plies = (int64_t)h[az::kStatPlies];
  st->errors = (int64_t)h[az::kStatErrors];
  st->evaluations = (int64_t)h[az::kStatNNEvals];
  st->cache_hits = (int64_t)h[az::kStatCacheHits];
  if (e->cache.ctl) {
    unsigned long long ctl[3];
    AZC_HIP(hipMemcpy(ctl, e->cache.ctl, sizeof(ctl), hipMemcpyDeviceToHost));
    st->cache_generation = (int64_t)ctl[0];
    st->cache_inserts = (int64_t)ctl[1];
    st->cache_entries = (int64_t)ctl[2];
    st->cache_gen_size = (int64_t)e->cache.gen_size;
    st->cache_capacity = (int64_t)e->cache.mask + 1;
  }
  st->issued_flop_per_board = e->net.use_tower && e->net.tower ? e->net.issued_flop_per_board : 0.0;
  st->tower_small_max_boards = -1;  // (chess: one tile height)
  st->active_slots = std::count_if(gid.begin(), gid.end(), [](int64_t v) { return v >= 0; });
  // conv-busy time = union of the timed conv intervals over all lanes
  std::vector<az::ConvTimer*> timers = {&e->timer};
  for (CLane* L : e->lanes) timers.push_back(&L->timer);
  std::vector<std::pair<double, double>> iv;
  for (az::ConvTimer* tm : timers) {
    tm->flush();
    st->conv_ms += tm->total_ms;
    st->conv_launches += tm->launches;
    iv.insert(iv.end(), tm->intervals.begin(), tm->intervals.end());
  }
  std::sort(iv.begin(), iv.end());
  double busy = 0.0, lo = 0.0, hi = -1.0;
  for (const auto& x : iv) {
    if (x.first > hi) {
      if (hi > lo) busy += hi - lo;
      lo = x.first;
      hi = x.second;
    } else {
      hi = std::max(hi, x.second);
    }
  }
  if (hi > lo) busy += hi - lo;
  st->conv_busy_ms = busy;
  return 0;
}

int az_chess_selfplay_step(az_chess_engine* e, int n_moves, az_stats* st) {
  if (!e || n_moves < 0) return az::fail_abi(AZ_E_INVALID, "bad arguments");
  if (!e->smp.done_count) return az::fail_abi(AZ_E_STATE, "az_chess_selfplay_begin was not called");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  const bool multi = e->lanes.size() > 1;
  for (int mv = 0; mv < n_moves; ++mv) {
    const int64_t m = e->moves_issued++;
    // lanes interleaved per simulation so every stream always has work queued
    for (int s = 0; s < e->g.sims; ++s)
      for (CLane* L : e->lanes)
        if ((rc = simulate(e, *L))) return rc;
    for (CLane* L : e->lanes)
      if ((rc = flush_expand(*L))) return rc;
    for (CLane* L : e->lanes) {
      // a lane plays move m once every other lane has finished move m - 1, so
      // move m - 1's games-finished snapshot holds no game of move m (the
      // drain's contract, as the Connect-N engine's)
      if (multi && m > e->batch_first_move)
        for (CLane* O : e->lanes)
          if (O != L) AZC_HIP(hipStreamWaitEvent(L->stream, O->move_done[(m - 1) % 4], 0));
      play_kernel<<<L->g.slots, 64, 0, L->stream>>>(L->g, L->t, e->smp, CPlayOut{});
      az::launch_move_end(e->move_arrive + m % 4, (int)e->lanes.size(), e->smp.done_count, e->snap_dev + m % 4,
                          L->stream);
      AZC_HIP(hipEventRecord(L->move_done[m % 4], L->stream));
    }
    AZC_HIP(hipGetLastError());
  }
  if (!st) return 0;  // asynchronous (ABI 10): the moves run on while the caller drains earlier ones
  if ((rc = sync_lanes(e))) return rc;
  if ((rc = check_errors(e))) return rc;
  return az_chess_stats(e, st);
}

int az_chess_selfplay_drain(az_chess_engine* e, int64_t max_games, int64_t* n_out, int64_t* game_ids,
                            int32_t* lengths, int32_t* results, int32_t* terminations, int32_t* expansions,
                            az_chess_pos* positions, uint16_t* moves, int32_t* policy_n, int16_t* policy_actions,
                            double* policy_probs) {
  if (!e || !n_out || max_games < 0) return az::fail_abi(AZ_E_INVALID, "bad arguments");
  *n_out = 0;
  if (!e->smp.done_count) return 0;  // no self-play batch begun
  AZC_HIP(hipSetDevice(e->device));
  // the newest move whose count snapshot is complete; if the last issued move
  // is still running, wait for the one before it (never for the running one)
  const int64_t last = e->moves_issued - 1;
  int64_t k = -1;
  bool last_done = last >= e->batch_first_move;
  if (last_done)
    for (CLane* L : e->lanes) last_done = last_done && hipEventQuery(L->move_done[last % 4]) == hipSuccess;
  if (last_done) {
    k = last;
  } else if (last - 1 >= e->batch_first_move) {
    k = last - 1;
    for (CLane* L : e->lanes) AZC_HIP(hipEventSynchronize(L->move_done[k % 4]));
  }
  if (k < 0) return 0;
  const unsigned long long done = __atomic_load_n(e->snap_host + k % 4, __ATOMIC_ACQUIRE);
  const int64_t n = std::min<int64_t>((int64_t)done - e->drained, max_games);
  if (n <= 0) return 0;
  // the finished games' ids, then each game's records (complete once its id
  // is listed: the play kernel stores them first); pack_stream holds nothing else
  std::vector<int64_t> ids((size_t)n);
  AZC_HIP(hipMemcpyAsync(ids.data(), e->smp.done_ids + e->drained, (size_t)n * sizeof(int64_t),
                         hipMemcpyDeviceToHost, e->pack_stream));
  AZC_HIP(hipStreamSynchronize(e->pack_stream));
  const CSamples& s = e->smp;
  const size_t P = (size_t)s.plies, M = AZ_CHESS_MAX_MOVES;
  hipStream_t q = e->pack_stream;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t gi = ids[(size_t)i] - s.first_game;
    if (gi < 0 || gi >= s.n_games) return az::fail_abi(AZ_E_STATE, "drained game id outside the batch");
    if (game_ids) game_ids[i] = ids[(size_t)i];
    if (lengths) AZC_HIP(hipMemcpyAsync(lengths + i, s.length + gi, sizeof(int32_t), hipMemcpyDeviceToHost, q));
    if (results) AZC_HIP(hipMemcpyAsync(results + i, s.result + gi, sizeof(int32_t), hipMemcpyDeviceToHost, q));
    if (terminations)
      AZC_HIP(hipMemcpyAsync(terminations + i, s.term + gi, sizeof(int32_t), hipMemcpyDeviceToHost, q));
    if (expansions)
      AZC_HIP(hipMemcpyAsync(expansions + i, s.expansions + gi, sizeof(int32_t), hipMemcpyDeviceToHost, q));
    if (positions)
      AZC_HIP(hipMemcpyAsync(positions + i * P, s.pos + gi * P, P * sizeof(az_chess_pos), hipMemcpyDeviceToHost, q));
    if (moves) AZC_HIP(hipMemcpyAsync(moves + i * P, s.moves + gi * P, P * sizeof(uint16_t), hipMemcpyDeviceToHost, q));
    if (policy_n)
      AZC_HIP(hipMemcpyAsync(policy_n + i * P, s.pol_n + gi * P, P * sizeof(int32_t), hipMemcpyDeviceToHost, q));
    if (policy_actions)
      AZC_HIP(hipMemcpyAsync(policy_actions + i * P * M, s.pol_a + gi * P * M, P * M * sizeof(int16_t),
                             hipMemcpyDeviceToHost, q));
    if (policy_probs)
      AZC_HIP(hipMemcpyAsync(policy_probs + i * P * M, s.pol_p + gi * P * M, P * M * sizeof(double),
                             hipMemcpyDeviceToHost, q));
  }
  AZC_HIP(hipStreamSynchronize(q));
  e->drained += n;
  *n_out = n;
  return 0;
}

int az_chess_selfplay_run(az_chess_engine* e, int64_t first_game, int64_t n_games, uint32_t base_seed,
                          az_stats* st) {
  int rc;
  if ((rc = az_chess_selfplay_begin(e, first_game, n_games, base_seed))) return rc;
  az_stats tmp;
  for (;;) {
    if ((rc = az_chess_selfplay_step(e, 1, &tmp))) return rc;
    if (tmp.active_slots == 0) break;
  }
  if (st) *st = tmp;
  return 0;
}

int az_chess_selfplay_results(az_chess_engine* e, int32_t* lengths, int32_t* results, int32_t* terminations,
                              int32_t* expansions, az_chess_pos* positions, uint16_t* moves, int32_t* policy_n,
                              int16_t* policy_actions, double* policy_probs) {
  if (!e) return az::fail_abi(AZ_E_INVALID, "null engine");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  if ((rc = sync_lanes(e))) return rc;
  const size_t G = (size_t)e->sp_n, P = (size_t)e->smp.plies, M = AZ_CHESS_MAX_MOVES;
  if (G == 0) return 0;
  const CSamples& s = e->smp;
  if (lengths) AZC_HIP(hipMemcpy(lengths, s.length, G * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (results) AZC_HIP(hipMemcpy(results, s.result, G * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (terminations) AZC_HIP(hipMemcpy(terminations, s.term, G * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (expansions) AZC_HIP(hipMemcpy(expansions, s.expansions, G * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (positions) AZC_HIP(hipMemcpy(positions, s.pos, G * P * sizeof(az_chess_pos), hipMemcpyDeviceToHost));
  if (moves) AZC_HIP(hipMemcpy(moves, s.moves, G * P * sizeof(uint16_t), hipMemcpyDeviceToHost));
  if (policy_n) AZC_HIP(hipMemcpy(policy_n, s.pol_n, G * P * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (policy_actions)
    AZC_HIP(hipMemcpy(policy_actions, s.pol_a, G * P * M * sizeof(int16_t), hipMemcpyDeviceToHost));
  if (policy_probs) AZC_HIP(hipMemcpy(policy_probs, s.pol_p, G * P * M * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

namespace {
int tree_buffers(az_chess_engine* e) {
  if (e->tree_move) return 0;
  const size_t S = (size_t)e->g.slots, M = AZ_CHESS_MAX_MOVES;
  int rc;
  if ((rc = e->alloc(&e->tree_u, S)) || (rc = e->alloc(&e->tree_status, S)) || (rc = e->alloc(&e->tree_pol_n, S)) ||
      (rc = e->alloc(&e->tree_slots, S)) || (rc = e->alloc(&e->tree_pol_a, S * M)) ||
      (rc = e->alloc(&e->tree_pol_p, S * M)) || (rc = e->alloc(&e->tree_roots, S)) ||
      (rc = e->alloc(&e->tree_move, S)))
    return rc;
  return 0;
}

int tree_slot_list(az_chess_engine* e, int n, const int32_t* slots) {
  if (n < 0 || n > e->g.slots || (n && !slots)) return az::fail_abi(AZ_E_INVALID, "bad slot list");
  std::vector<char> seen(e->g.slots, 0);
  for (int i = 0; i < n; ++i) {
    if (slots[i] < 0 || slots[i] >= e->g.slots || seen[slots[i]])
      return az::fail_abi(AZ_E_INVALID, "slot index out of range or repeated");
    seen[slots[i]] = 1;
  }
  int rc;
  if ((rc = tree_buffers(e))) return rc;
  if (n) AZC_HIP(hipMemcpyAsync(e->tree_slots, slots, n * sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
  return 0;
}
}  // namespace

int az_chess_tree_reset(az_chess_engine* e, int n, const int32_t* slots, const az_chess_pos* roots) {
  if (!e || (n && !roots)) return az::fail_abi(AZ_E_INVALID, "null argument");
  if (e->cfg.evaluator == AZ_EVAL_NETWORK && !e->net.ready)
    return az::fail_abi(AZ_E_STATE, "network evaluator selected but az_chess_engine_set_weights was not called");
  AZC_HIP(hipSetDevice(e->device));
  for (CLane* L : e->lanes) L->pending_expand = false;  // (a search an error interrupted)
  int rc;
  if ((rc = sync_lanes(e)) || (rc = tree_slot_list(e, n, slots))) return rc;
  if (!n) return 0;
  // a root must be a position the device rules accept (legal move list fits)
  std::vector<az_chess_pos> r(roots, roots + n);
  for (const az_chess_pos& p : r)
    if (p.turn > 1 || p.ep_square < -1 || p.ep_square > 63)
      return az::fail_abi(AZ_E_INVALID, "malformed az_chess_pos");
  AZC_HIP(hipMemcpyAsync(e->tree_roots, r.data(), n * sizeof(az_chess_pos), hipMemcpyHostToDevice, e->stream));
  tree_reset_kernel<<<(n + 63) / 64, 64, 0, e->stream>>>(e->g, e->t, n, e->tree_slots, e->tree_roots);
  AZC_HIP(hipGetLastError());
  AZC_HIP(hipStreamSynchronize(e->stream));
  return 0;
}

int az_chess_tree_release(az_chess_engine* e, int n, const int32_t* slots) {
  if (!e) return az::fail_abi(AZ_E_INVALID, "null engine");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  if ((rc = sync_lanes(e)) || (rc = tree_slot_list(e, n, slots))) return rc;
  if (!n) return 0;
  tree_release_kernel<<<(n + 63) / 64, 64, 0, e->stream>>>(e->t, n, e->tree_slots);
  AZC_HIP(hipGetLastError());
  AZC_HIP(hipStreamSynchronize(e->stream));
  return 0;
}

int az_chess_tree_search(az_chess_engine* e, int n_sims) {
  if (!e || n_sims < 0) return az::fail_abi(AZ_E_INVALID, "bad arguments");
  if (e->cfg.evaluator == AZ_EVAL_NETWORK && !e->net.ready)
    return az::fail_abi(AZ_E_STATE, "network evaluator selected but az_chess_engine_set_weights was not called");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  for (int s = 0; s < n_sims; ++s)
    for (CLane* L : e->lanes)
      if ((rc = simulate(e, *L))) return rc;
  for (CLane* L : e->lanes)
    if ((rc = flush_expand(*L))) return rc;
  if ((rc = sync_lanes(e))) return rc;
  return check_errors(e);
}

int az_chess_tree_play(az_chess_engine* e, const double* uniforms, int greedy, int deterministic, int32_t* moves,
                       int32_t* status, int32_t* policy_n, int16_t* policy_actions, double* policy_probs) {
  if (!e || (!deterministic && !uniforms)) return az::fail_abi(AZ_E_INVALID, "bad arguments");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  if ((rc = sync_lanes(e)) || (rc = tree_buffers(e))) return rc;
  const size_t S = (size_t)e->g.slots, M = AZ_CHESS_MAX_MOVES;
  if (!deterministic) AZC_HIP(hipMemcpyAsync(e->tree_u, uniforms, S * sizeof(double), hipMemcpyHostToDevice, e->stream));
  AZC_HIP(hipMemsetAsync(e->tree_move, 0xff, S * sizeof(int32_t), e->stream));
  AZC_HIP(hipMemsetAsync(e->tree_status, 0, S * sizeof(int32_t), e->stream));
  AZC_HIP(hipMemsetAsync(e->tree_pol_n, 0, S * sizeof(int32_t), e->stream));
  AZC_HIP(hipStreamSynchronize(e->stream));
  for (CLane* L : e->lanes) {
    const size_t f = (size_t)L->first;
    CPlayOut po;
    po.uniforms = deterministic ? nullptr : e->tree_u + f;
    po.greedy = greedy ? 1 : 0;
    po.deterministic = deterministic ? 1 : 0;
    po.move = e->tree_move + f;
    po.status = e->tree_status + f;
    po.pol_n = e->tree_pol_n + f;
    po.pol_a = e->tree_pol_a + f * M;
    po.pol_p = e->tree_pol_p + f * M;
    play_kernel<<<L->g.slots, 64, 0, L->stream>>>(L->g, L->t, CSamples{}, po);
  }
  AZC_HIP(hipGetLastError());
  if ((rc = sync_lanes(e)) || (rc = check_errors(e))) return rc;
  if (moves) AZC_HIP(hipMemcpy(moves, e->tree_move, S * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (status) AZC_HIP(hipMemcpy(status, e->tree_status, S * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (policy_n) AZC_HIP(hipMemcpy(policy_n, e->tree_pol_n, S * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (policy_actions) AZC_HIP(hipMemcpy(policy_actions, e->tree_pol_a, S * M * sizeof(int16_t), hipMemcpyDeviceToHost));
  if (policy_probs) AZC_HIP(hipMemcpy(policy_probs, e->tree_pol_p, S * M * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int az_chess_tree_info(az_chess_engine* e, int slot, int64_t* info, float* root_value) {
  if (!e || !info || slot < 0 || slot >= e->g.slots) return az::fail_abi(AZ_E_INVALID, "bad arguments");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  if ((rc = sync_lanes(e))) return rc;
  int32_t top, first, cnt, ply;
  int64_t gid;
  AZC_HIP(hipMemcpy(&top, e->t.top + slot, 4, hipMemcpyDeviceToHost));
  AZC_HIP(hipMemcpy(&first, e->t.root_first + slot, 4, hipMemcpyDeviceToHost));
  AZC_HIP(hipMemcpy(&cnt, e->t.root_n + slot, 4, hipMemcpyDeviceToHost));
  AZC_HIP(hipMemcpy(&ply, e->t.ply + slot, 4, hipMemcpyDeviceToHost));
  AZC_HIP(hipMemcpy(&gid, e->t.game_id + slot, 8, hipMemcpyDeviceToHost));
  if (root_value) AZC_HIP(hipMemcpy(root_value, e->t.root_value + slot, 4, hipMemcpyDeviceToHost));
  info[0] = top;
  info[1] = first;
  info[2] = cnt;
  info[3] = ply;
  info[4] = gid >= 0;
  return 0;
}

int az_chess_tree_export(az_chess_engine* e, int slot, double* prior, double* w, int32_t* n, int32_t* child,
                         int32_t* child_n, int32_t* moves, float* child_value) {
  if (!e || slot < 0 || slot >= e->g.slots) return az::fail_abi(AZ_E_INVALID, "bad arguments");
  AZC_HIP(hipSetDevice(e->device));
  int rc;
  if ((rc = sync_lanes(e))) return rc;
  int32_t top, half;
  AZC_HIP(hipMemcpy(&top, e->t.top + slot, 4, hipMemcpyDeviceToHost));
  AZC_HIP(hipMemcpy(&half, e->t.half + slot, 4, hipMemcpyDeviceToHost));
  std::vector<az::Edge> h(top);
  if (top)
    AZC_HIP(hipMemcpy(h.data(), e->t.edges + ((size_t)slot * 2 + half) * e->g.half_cap, top * sizeof(az::Edge),
                      hipMemcpyDeviceToHost));
  for (int i = 0; i < top; ++i) {
    if (prior) prior[i] = h[i].prior;
    if (w) w[i] = h[i].W;
    if (n) n[i] = h[i].N;
    if (child) child[i] = h[i].child;
    if (child_n) child_n[i] = h[i].child_n;
    if (moves) moves[i] = (uint16_t)h[i].action;
    if (child_value) child_value[i] = h[i].child_value;
  }
  return 0;
}

int az_chess_timer_enable(az_chess_engine* e, int on) {
  if (!e) return az::fail_abi(AZ_E_INVALID, "null engine");
  AZC_HIP(hipSetDevice(e->device));
  AZC_HIP(hipStreamSynchronize(e->stream));
  if (!e->timer_ref) AZC_HIP(hipEventCreate(&e->timer_ref));
  AZC_HIP(hipEventRecord(e->timer_ref, e->stream));
  AZC_HIP(hipStreamSynchronize(e->stream));
  int rc;
  if ((rc = sync_lanes(e))) return rc;
  std::vector<az::ConvTimer*> timers = {&e->timer};
  for (CLane* L : e->lanes) timers.push_back(&L->timer);
  for (az::ConvTimer* tm : timers) {
    tm->flush();
    tm->reset();
    tm->ref = &e->timer_ref;
    tm->enabled = on != 0;
  }
  return 0;
}

}  // extern "C"
