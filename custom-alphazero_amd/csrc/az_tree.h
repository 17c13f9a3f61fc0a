// az_tree.h -- device-resident MCTS forest: one tree per game slot.
#pragma once
#include "az_device.h"

namespace az {

// One tree edge (reference UCTEdge, mcts/mcts.py:22-33) = 32 bytes.  A node
// is implicit: the contiguous run of edges its expansion allocated.  Child
// boards are not stored; select() replays the path's moves from the root
// board (board rules are cheap, HBM bytes are not).
struct Edge {
  double W;           // total_action_value (float64, += in path order)
  double prior;       // float32 prior widened exactly, or the float64 1/n uniform
  int32_t N;          // visit_count
  int32_t child;      // first edge of the child's expansion, kNoChild if leaf
  int16_t child_n;    // child's edge count (0 = unexpanded or terminal)
  int16_t action;     // index into all_possible_moves
  float child_value;  // child's evaluated_value (tree export only)
};
static_assert(sizeof(Edge) == 32, "Edge must stay 32 bytes");

// Counters/stat words (unsigned long long, device), each on a 128-byte line
// of its own (kStatStride words apart): every wave of every lane adds to them
// (wave-aggregated atomics), and counters sharing a line serialised in its
// L2 channel (round 6).  An index below is the word offset of its counter.
constexpr int kStatStride = 16;
enum : int {
  kStatExpansions = 0 * kStatStride,   // evaluate_and_expand calls
  kStatTerminal = 1 * kStatStride,     // terminal leaf visits
  kStatGamesDone = 2 * kStatStride,
  kStatErrors = 3 * kStatStride,       // bit flags below
  kStatSims = 4 * kStatStride,         // per-slot simulations
  kStatPlies = 5 * kStatStride,
  kStatNextGame = 6 * kStatStride,     // next game id to hand to a free slot
  kStatCacheHits = 7 * kStatStride,    // expansions served by the transposition cache
  kStatNNEvals = 8 * kStatStride,      // boards the evaluator actually computed
  kStatCacheInserts = 9 * kStatStride,
  kStatPathEdges = 10 * kStatStride,   // edges on the selected paths (sum of select depths)
  kStatMaxRetained = 11 * kStatStride, // compaction: most edges kept (atomicMax)
  kStatPoolHigh = 12 * kStatStride,    // pooled arenas: most edges a lane's half held at a move's end (atomicMax)
  kStatCount = 13 * kStatStride        // words (kStatCacheInserts counts since engine creation; CacheDev::ctl since a clear)
};
// a lane's per-simulation queue counters (eval, miss, nn, dup), one block per
// simulation parity, each counter on a 128-byte line of its own
constexpr int kCountStride = 32;
constexpr int kCountWords = 2 * 4 * kCountStride;
enum : unsigned long long {
  kErrArena = 1, kErrPow = 2, kErrPath = 4, kErrIllegal = 8, kErrNoRoot = 16,
  kErrActRange = 32,  // a conv16 activation beyond the split16 range (|x| > 32752)
  kErrNoise = 64      // the tree API's host-drawn root noise ran out of rows
};

// All device state of a forest (struct of arrays over slots).
//
// Arenas.  halves == 1 (the tree API, uncompacted self-play): slot s owns the
// static run edges[s * arena_cap, (s + 1) * arena_cap); edge indices are
// relative to it.  halves == 2 (compacted self-play): every lane owns a POOL
// of two halves of pool_cap edges; a move's search allocates from the
// current half (`edges`, bump counter `pool_top`) in chunks of kPoolChunkA * A
// edges per slot, and compaction copies each slot's kept subtree into the
// other half (`dst_edges`, `dst_top`), reserving the slot's live edge count
// there in one bump.  After a lane's compaction the current half is empty:
// its counter resets and the halves swap (host side, the next launches'
// views).  Edge indices are pool-half indices.  The pool is shared by the
// lane's slots, so one game whose kept subtree grows large (a peaked
// network) borrows what other slots do not use; overflow raises kErrArena.
constexpr int kPoolChunkA = 16;
struct TreeDev {
  Edge* edges;                 // halves == 1: [slots][arena_cap]; 2: the lane's current pool half
  int32_t* arena_end;          // [slots] pool: end of the slot's current chunk
  int32_t* slot_live;          // [slots] pool: edges of the slot's tree in the current half
  unsigned long long* pool_top;  // pool: the current half's bump counter
  Edge* dst_edges;             // pool: the other half (compaction target) ...
  unsigned long long* dst_top;   // ... and its counter
  int32_t pool_cap;            // pool: edges per half
  Board* root_board;           // [slots]
  int32_t* root_first;         // [slots]
  int32_t* root_n;             // [slots]
  float* root_value;           // [slots]
  int32_t* arena_top;          // [slots] next free edge (static: of the slot's run; pool: of the half)
  int32_t* ply;                // [slots] (Board.fullmove_number)
  int64_t* game_id;            // [slots], -1 = idle
  int32_t* path;               // [slots][max_depth]
  int32_t* path_len;           // [slots]
  int32_t* slot_expansions;    // [slots], this game's expansions so far
  uint32_t* mt;                // [625][mt_stride], word-major MT19937 state (+ index)
  int32_t mt_stride;           // slots of the whole engine (a lane view offsets mt)
  // the slot's leaf of this simulation, read by the expand launch (one
  // thread per slot): (leaf_epoch << 32) | src, src >= 0 a cache entry, < 0
  // -(evaluator row + 1); another simulation's tag: no leaf (idle, terminal)
  uint64_t* leaf_src;          // [slots]
  Board* leaf_board;           // [slots]
  uint32_t leaf_epoch;         // this simulation's tag, unique over the engine's lanes
  Board* eval_board;           // [slots] evaluator rows with the cache off (every leaf)
  int32_t* eval_count;         // [1]
  int32_t* miss_count;         // [1]
  Board* nn_board;             // [slots] evaluator rows with the cache on (the misses)
  int32_t* nn_count;           // [1]
  // eval/miss/nn counts (and a spare word) are one block of 4; two blocks
  // alternate by simulation (epoch parity): the select kernel zeroes the
  // other block, the next simulation's, so no memset launch sits between
  int32_t* next_counts;        // [4 * kCountStride] the block the next simulation uses
  uint32_t epoch;              // the lane's simulation counter (its parity picks the block)
  unsigned long long* stats;   // [kStatCount]
  const double* powtab;        // [pow_len]: libm pow(n, 0.5), host-built
  // per-move outputs (MCTS API play())
  int32_t* last_move;          // [slots] action played (-1 none)
  int32_t* last_status;        // [slots] 0 ongoing / 1 win / 2 draw
  double* last_policy;         // [slots][A]
  // tree API root noise drawn by the host (az_tree_search_noise): slot s's
  // r-th root selection of the search mixes noise_in[(s * noise_rows + r) * A + i]
  // into edge i's prior; null: self-play draws on the device from the slot's MT19937
  const double* noise_in;
  int32_t* noise_cur;          // [slots] rows consumed
  int32_t noise_rows;
};

// Transposition cache = the reference's plays_inferences (mcts/mcts.py:122-143,
// utils.py:38-39): board -> (probs[A], value), shared by every game on the
// device, cleared when the weights change.  Set-associative: a board hashes
// to one bucket of kCacheBucket slots (its state words are one 64-B segment,
// read in one round trip); inserts take the bucket's first reusable slot and
// are dropped when every slot is live.  (Round 2 probed linearly across the
// table: once stale entries had filled it, a miss walked max_probe = 32
// acquire loads one after another, and games/s fell the longer a run went.)
// The evaluator is deterministic per board, so hits never change a search.
//
// Eviction: least recently used, by generations (the reference's dict grows
// without bound until the next model; a fixed table keeps what it can).
// Every Ready entry is live -- a lookup accepts any of them, so the whole
// table serves as plays_inferences.  Each `gen_size` inserts start a new
// generation; a hit on an entry of an older generation moves it into the
// current one (one CAS per entry per generation), so an entry's generation
// is when it was last used.  An insert takes the bucket's first empty slot,
// else its least recently used entry at least kCacheEvictAge generations old
// (dropped when every entry is younger: a bucket of boards all in use).
//
// Overwrite safety: select finds an entry and expand reads its payload one
// launch later.  Every hit leaves select stamped with the reader's generation
// G (an older entry's refresh CAS must win; when it loses, the slot may be
// being overwritten and the board counts as a miss).  The engine enables
// eviction only when gen_size exceeds three moves of every slot's inserts
// (slots * sims * 3: the lane drift is bounded to two moves by move events,
// az_engine.hip), so at most one generation turn falls inside a reader's
// window, an insert sees the entry at most 1 generation old, and
// kCacheEvictAge = 2 keeps it.
//
// State word: [31:16] 16-bit fingerprint (hash bits 48-63, so most probes
// need no key read), [15:2] generation mod 2^14, [1:0] status.
enum : uint32_t { kCacheEmpty = 0, kCacheClaimed = 1, kCacheReady = 2 };
constexpr uint32_t kCacheGenMask = 0x3fff;
constexpr uint32_t kCacheGenDiv = 16;   // a generation = capacity / kCacheGenDiv inserts
constexpr uint32_t kCacheEvictAge = 2;  // an insert may overwrite entries this many generations old
AZ_HD uint32_t cache_fp(uint64_t h) { return (uint32_t)(h >> 48); }
AZ_HD uint32_t cache_age(uint32_t st, uint32_t gen) { return (gen - (st >> 2)) & kCacheGenMask; }
AZ_HD uint32_t cache_word(uint32_t fp, uint32_t gen, uint32_t status) {
  return (fp << 16) | ((gen & kCacheGenMask) << 2) | status;
}
struct CacheDev {
  Board* keys = nullptr;       // [cap]
  uint32_t* state = nullptr;   // [cap]
  float* pay = nullptr;        // [cap][A+1]: probs then value
  uint32_t mask = 0;           // cap - 1
  int enabled = 0;
  unsigned long long* ctl = nullptr;  // device [0] generation, [1] inserts since the last clear,
                                      // [2] of them into empty slots (= entries held)
  unsigned long long gen_size = 0;    // inserts per generation; 0 = no eviction
};
constexpr int kCacheBucket = 16;  // slots per bucket (cache_log2 >= 4)
AZ_HD uint32_t cache_bucket(const CacheDev& c, uint64_t h) {
  return (uint32_t)h & c.mask & ~(uint32_t)(kCacheBucket - 1);
}

// Self-play sample sink, indexed by game id - first_game.
struct SampleDev {
  int64_t first_game = 0, n_games = 0;
  uint32_t base_seed = 0;
  Board* boards = nullptr;     // [n_games][max_plies]: root board before each move
  double* policy = nullptr;    // [n_games][max_plies][A]
  int16_t* moves = nullptr;    // [n_games][max_plies]
  int32_t* length = nullptr;   // [n_games]
  int32_t* result = nullptr;   // [n_games]: get_result(keep_same_player=True)
  int32_t* expansions = nullptr;  // [n_games]
  int64_t* done_ids = nullptr;    // [n_games] game ids in the order they finished
  unsigned long long* done_count = nullptr;  // [1]
};

// Finished games [from, from + n) of smp.done_ids packed for one D2H copy
// (az_selfplay_drain): ids, lengths, results, expansions, then per game
// HW plies of int8 cells (row-major, canonical), f64 policies [HW][A] and
// int16 moves.  Layout of one record: drain_record_bytes().
size_t drain_record_bytes(const GameCfg& g);
void launch_drain_pack(const GameCfg& g, const SampleDev& smp, int64_t from, int n, uint8_t* out,
                       hipStream_t s);

// the base edge indices of slot s are relative to
AZ_HD Edge* slot_edges(const GameCfg& g, const TreeDev& t, int s) {
  return g.halves > 1 ? t.edges : t.edges + (size_t)s * g.arena_cap;
}

void launch_select(const GameCfg& g, const TreeDev& t, const CacheDev& c, hipStream_t s);
// self-play tree reuse (halves == 2): the new root's subtree into the other
// pool half; then the current half's counter is reset (its high-water mark to
// kStatPoolHigh) -- the host swaps the halves for the next move
void launch_compact(const GameCfg& g, const TreeDev& t, hipStream_t s);
// end of a lane's move: the last of n_lanes lanes to arrive stores the
// games-finished count into *snap (pinned host memory) and resets *arrive
void launch_move_end(int32_t* arrive, int n_lanes, const unsigned long long* done_count,
                     unsigned long long* snap, hipStream_t s);
// cache on: misses are deduplicated inside select (step tag table); this
// resolves the ones whose tag matched, by full-board compare
void launch_synth_eval(const GameCfg& g, const Board* boards, const int32_t* count, float* probs,
                       float* values, hipStream_t s);
void launch_expand(const GameCfg& g, const TreeDev& t, const CacheDev& c, const float* probs,
                   const float* values, hipStream_t s);
// uniforms: device [slots] draws for play (MCTS API), or null -> per-slot MT19937;
// greedy_mode -1 = by ply (self-play), 0/1 = caller's flag
void launch_play(const GameCfg& g, const TreeDev& t, const SampleDev& smp, const double* uniforms,
                 int greedy_mode, int deterministic, int refill, hipStream_t s);
void launch_slot_init(const GameCfg& g, const TreeDev& t, const SampleDev& smp, int64_t n_first,
                      hipStream_t s);
void launch_slot_release(const TreeDev& t, const int32_t* slots, int n, hipStream_t s);
void launch_slot_set_root(const GameCfg& g, const TreeDev& t, const int32_t* slots,
                          const Board* boards, int n, hipStream_t s);

}  // namespace az
