/*
 * az.h -- C ABI of libaz, the MI355X (gfx950) self-play engine.
 *
 * The reference (neuronest/custom-alphazero) is Python: its plug-in seams are
 * duck-typed calls, not an FFI.  Each entry point below replaces one of those
 * seams; the Python drop-in package (custom-alphazero_amd/custom_alphazero)
 * binds them with ctypes (INTEGRATION.md shows the binding).  Paths are
 * relative to the reference root.
 *
 * Conventions: every function returns 0 on success or a negative AZ_E* code;
 * az_last_error() then holds a thread-local message.  Host buffers are owned
 * by the caller; the engine owns all device memory.  One engine = one device;
 * calls are synchronous (results are in the caller's buffers on return),
 * except az_selfplay_step without stats and az_selfplay_drain, which run
 * beside the queued moves -- every other call that touches engine buffers
 * first waits for them.  No exception or abort crosses the ABI.
 */
#ifndef AZ_H_
#define AZ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AZ_ABI_VERSION 10

#define AZ_OK 0
#define AZ_E_INVALID -1  /* bad argument / config */
#define AZ_E_HIP -2      /* HIP runtime error */
#define AZ_E_STATE -3    /* call out of order (e.g. no weights) */
#define AZ_E_DEVICE -4   /* a kernel flagged an error (arena/pow/path overflow, activation range) */
#define AZ_E_CALLBACK -5 /* the host evaluator (AZ_EVAL_HOST) returned nonzero */

#define AZ_EVAL_NETWORK 0    /* the policy/value network (model/tensorflow/model.py) */
#define AZ_EVAL_SYNTHETIC 1  /* oracle/synth.py's exact evaluator (parity runs) */
#define AZ_EVAL_HOST 2       /* a host callback (az_engine_set_evaluator): the reference's
                                duck-typed self.model(x) seam, mcts/mcts.py:130-137 */

/* az_config.conv_algo */
#define AZ_CONV_F16X2 0      /* direct implicit GEMM on the fp16 MFMA, fp32-accurate: both operands
                                as two fp16 terms, three products per k-step (default); Connect-N
                                runs the whole forward in one kernel, activations held in LDS */
#define AZ_CONV_DIRECT 1     /* direct implicit GEMM on fp32 MFMA (exact fp32 FMA chains) */
#define AZ_CONV_F16X2_LAYERS 2  /* AZ_CONV_F16X2's arithmetic one layer per launch (activations in
                                   HBM between layers; the round-2 path, kept for A/B runs) */

typedef struct az_engine az_engine;

/* Engine configuration: the reference's Config* class constants
 * (custom_alphazero/config.py:7-71) plus device sizing. */
typedef struct az_config {
    int32_t board_height;          /* ConfigConnectN.board_height (config.py:40) */
    int32_t board_width;           /* ConfigConnectN.board_width (config.py:39) */
    int32_t n;                     /* ConfigConnectN.n (config.py:41) */
    int32_t gravity;               /* ConfigConnectN.gravity (config.py:42) */
    int32_t mcts_iterations;       /* sims per move: ConfigSelfPlay.mcts_iterations (config.py:21) */
    int32_t index_move_greedy;     /* ConfigMCTS.index_move_greedy (config.py:55) */
    double exploration_constant;   /* ConfigMCTS.exploration_constant (config.py:51) */
    int32_t slots;                 /* concurrent games (trees) on this device */
    int32_t evaluator;             /* AZ_EVAL_* */
    int32_t filters;               /* ConfigModel.filters (config.py:71); 128 supported */
    int32_t depth;                 /* ConfigModel.depth (config.py:63) */
    int32_t value_hidden;          /* ValueHead hidden_dim (model/tensorflow/model.py:110) */
    double bn_epsilon;             /* Keras BatchNormalization epsilon (1e-3) */
    int64_t arena_edges;           /* tree edges per slot (compact: the average per slot of a lane's
                                      pooled halves); 0 = mcts_iterations*H*W*A + A, no game can
                                      overflow it */
    int64_t max_tree_visits;       /* bound on visits through one node; 0 = mcts_iterations*H*W */
    int32_t cache_log2;            /* transposition cache entries = 2^cache_log2 (the reference's
                                      plays_inferences, mcts/mcts.py:122-143); 0 = off, else 4..30
                                      (16-slot buckets) */
    int32_t conv_algo;             /* residual-tower 3x3 convs: AZ_CONV_F16X2 (0, default; depth <= 16,
                                      value_hidden <= 256), AZ_CONV_DIRECT (1) or AZ_CONV_F16X2_LAYERS
                                      (2; board width <= 16, activations within +-32752); same
                                      layer, outputs within NET_TOL */
    int32_t lanes;                 /* self-play slot groups searched on separate HIP streams
                                      (0 = auto: 2 when slots >= 512); results do not depend on it */
    int32_t compact;               /* 1: after every self-play move the chosen child's subtree is
                                      copied into the other half of the lane's pooled arena (the
                                      subtrees the game has left are reclaimed, mcts.py:207).  Each
                                      lane (slot group) owns two halves of arena_edges x its slots
                                      edges; a slot takes 16*A-edge chunks of the current half as it
                                      expands, so the slots share the room (0 = the overflow-proof
                                      size S*H*W*A + A per slot, or, when two such halves per slot
                                      exceed 40% of the free HBM, the most that fits there and at
                                      least 8*mcts_iterations*A + H*W*A; overflow is AZ_E_DEVICE).
                                      The tree API (az_tree_*) does not compact: it refuses such an
                                      engine */
    int32_t tower_natural_order;   /* 1: the one-launch tower computes its tiles in natural pixel order
                                      (no slot plan, no skipped edge taps): bitwise the same outputs
                                      (tests, A/B runs); 0 = the slot plan (default) */
    int32_t dirichlet_noise;       /* ConfigMCTS.enable_dirichlet_noise (config.py:52): every root
                                      selection mixes the priors with a fresh Dirichlet draw
                                      (mcts.py:70-85, :115-116) -- in self-play from the game's
                                      MT19937 stream, in the tree API the caller's draws
                                      (az_tree_search_noise) */
    double dirichlet_alpha;        /* ConfigMCTS.dirichlet_noise_value (config.py:53, 0.03) */
    double dirichlet_ratio;        /* ConfigMCTS.dirichlet_noise_ratio (config.py:54, 0.25) */
    int32_t rng_skip;              /* MT19937 words each self-play game's stream discards after seeding
                                      (ABI 9): the reference's play_game seeds np.random, then builds
                                      the model, whose constructor draws np.random.rand(1, H, W, 4)
                                      (self_play.py:45-47, model/tensorflow/model.py:167-169): 2*H*W*4
                                      words.  0 = none */
    int32_t reserved[1];
} az_config;

/* One named weight tensor in Keras layout ("Weights"). */
typedef struct az_tensor {
    const char* name;   /* e.g. "block0.conv1.kernel" */
    const float* data;  /* host pointer, or device pointer when on_device = 1 */
    int64_t numel;
    int32_t on_device;
    int32_t reserved;
} az_tensor;

typedef struct az_stats {
    int64_t expansions;       /* evaluate_and_expand calls (mcts/mcts.py:145) */
    int64_t terminal_visits;  /* leaves that were game-over (mcts.py:176-179) */
    int64_t games_done;
    int64_t simulations;      /* per-tree simulations executed */
    int64_t plies;            /* moves committed */
    int64_t active_slots;     /* slots still holding a game */
    int64_t errors;           /* device error flags (0 = none) */
    int64_t conv_launches;    /* timed conv kernels (az_timer_enable) */
    double conv_ms;           /* their summed device time */
    int64_t cache_hits;       /* expansions served by the transposition cache */
    int64_t evaluations;      /* boards the evaluator computed (network or synthetic) */
    double conv_busy_ms;      /* union of the timed conv intervals over all lanes (device
                                 time in which at least one lane's conv kernels ran) */
    int64_t tree_launches;    /* timed select + expand kernels (az_timer_enable) */
    double tree_ms;           /* their summed device time */
    int64_t path_edges;       /* edges on the selected paths (sum of select depths) */
    int64_t cache_inserts;    /* transposition-cache inserts since the last clear */
    int64_t cache_generation; /* eviction generations since the last clear (az_tree.h: a generation is
                                 cache_gen_size inserts, an entry's stamp is its last use) */
    int64_t cache_gen_size;   /* inserts per generation (0 = no eviction: the table only fills) */
    int64_t cache_capacity;   /* cache entries (2^cache_log2; 0 = no cache) */
    int64_t games_drained;    /* finished games az_selfplay_drain has returned this batch */
    int64_t max_retained;     /* compact: most edges a compaction kept (the arena high-water mark
                                 before the next search) since engine creation */
    int64_t cache_entries;    /* entries the cache holds (every one is looked up: a hit moves it into
                                 the current generation, an insert into a full bucket evicts its least
                                 recently used entry 2+ generations old; ABI 10, was cache_live_gens) */
    int64_t arena_edges;      /* tree edges per slot this engine allocated (compact: per half, the
                                 average over a lane's pool) */
    double issued_flop_per_board; /* MFMA FLOP the network forward issues per board (the one-launch
                                     tower: per full tile after its slot plan's skipped taps, / boards
                                     per tile; 0 = not reported).  Chess (az_chess_stats): the
                                     self-play forward's, whose stem skips the always-zero history
                                     planes 0-63; az_chess_forward runs every plane: 18 more
                                     k-steps of 96 MFMAs (28.3 MFLOP) per board */
    int64_t arena_pool_edges; /* compact: edges of every lane's two pool halves (0 uncompacted) */
    int64_t arena_pool_high;  /* compact: most edges one lane's half held at a move's end */
    double issued_flop_per_board_small; /* the dual tower launch's smaller tiles (Connect-4: 96 rows of
                                           two boards), which a launch runs when it holds at most
                                           tower_small_max_boards live boards; 0 = no dual launch */
    int64_t tower_small_max_boards;     /* that threshold (2 x CUs / lanes; -1 = no dual launch) */
} az_stats;

int az_abi_version(void);
const char* az_last_error(void);
/* Build identity: a hash of the sources libaz was compiled from (profiles
 * record it, bench.py matches it), and the extra compile flags of a
 * diagnostic build (empty for the product library). */
const char* az_build_id(void);
const char* az_build_flags(void);

/* Replaces constructing PolicyValueModel + MCTS per game
 * (self_play.py:46-57, utils.py:42-48). */
int az_engine_create(int device, const az_config* cfg, az_engine** out);
int az_engine_destroy(az_engine* eng);
/* The number of slot groups (streams) the engine runs: az_config.lanes, or
 * for lanes = 0 the engine's choice -- 1 below 512 slots; 3 for 1536-4096
 * slots when the process has at least 8 HIP hardware queues
 * (GPU_MAX_HW_QUEUES as the environment held it when libaz loaded -- HIP reads
 * it once at its initialisation; the Python package sets 8 at import: a queue
 * per lane stream; configs[1] +4.9% games/s over
 * 2); else 2. */
int az_engine_lanes(const az_engine* eng);

/* Replaces PolicyValueModel.load_with_meta / set_weights
 * (model/tensorflow/model.py:190-201): the engine copies and folds them. */
int az_engine_set_weights(az_engine* eng, const az_tensor* tensors, int n);

/* AZ_EVAL_HOST: the evaluator the search calls once per simulation (and
 * lane) with the leaves that need an evaluation -- after the transposition
 * cache and per-simulation dedup, so each board at most once -- as x
 * [n][H][W][4] f32 full_state planes (connect_n/board.py:83-98); it writes
 * the model's raw outputs probs [n][A] (before the legal-move mask and
 * renormalisation, mcts.py:147-150) and values [n], and returns 0 (nonzero:
 * the search fails with AZ_E_CALLBACK, and the simulation it interrupted
 * leaves the trees incomplete: az_selfplay_step, az_tree_search and
 * az_tree_play then fail with AZ_E_STATE until az_selfplay_begin or
 * az_tree_reset).  Host buffers, valid during the call.
 * The outputs must be a deterministic function of the board (the cache
 * relies on it, as the reference's plays_inferences dict does). */
typedef int32_t (*az_eval_fn)(void* user, const float* x, int32_t n, float* probs, float* values);
int az_engine_set_evaluator(az_engine* eng, az_eval_fn fn, void* user);

/* Board.full_state + Board.legal_moves_mask for a batch of canonical int8
 * boards [n][H][W] (connect_n/board.py:91-98, :154-155) -> state
 * [n][H][W][4] f32, mask [n][A] u8.  Either output may be NULL. */
int az_encode(az_engine* eng, const int8_t* boards, int n, float* state, uint8_t* mask);

/* PolicyValueModel.__call__ (model/tensorflow/model.py:182-188): x [n][H][W][4]
 * f32 -> probs [n][A] f32, values [n] f32.  Host buffers. */
int az_forward(az_engine* eng, const float* x, int n, float* probs, float* values);

/* Batched self_play.play / play_game (self_play.py:37-119): games
 * first_game .. first_game+n_games-1, game g seeded with MT19937(base_seed+g)
 * (the reference seeds np.random per game, self_play.py:45), slots refilled
 * as games end.  begin+step lets a caller time a window of moves; run does
 * begin + steps until every game is done.  step with st = NULL only enqueues
 * the moves and returns (no synchronize, device errors surface at the next
 * synchronizing call); with st it waits for them and fills the stats. */
int az_selfplay_begin(az_engine* eng, int64_t first_game, int64_t n_games, uint32_t base_seed);
int az_selfplay_step(az_engine* eng, int n_moves, az_stats* st);
int az_selfplay_run(az_engine* eng, int64_t first_game, int64_t n_games, uint32_t base_seed,
                    az_stats* st);
/* Per game g (index from first_game): lengths[g] plies; results[g] =
 * get_result(keep_same_player=True) of the final board (1 win, 0 draw);
 * expansions[g]; boards [g][H*W][H][W] int8 canonical root before each move;
 * policies [g][H*W][A] f64 (MCTS.play return_details policy); moves [g][H*W]. */
int az_selfplay_results(az_engine* eng, int32_t* lengths, int32_t* results, int32_t* expansions,
                        int8_t* boards, double* policies, int32_t* moves);
/* The games that finished since the previous drain (at most max_games, in the
 * order they finished), copied to the caller's buffers: the batch's samples
 * reach the host while self-play continues (play()'s results return,
 * self_play.py:112-118, one step at a time).  *n_out = games copied; per game
 * i: game_ids[i], lengths/results/expansions[i] as az_selfplay_results,
 * boards [i][H*W][H][W] int8, policies [i][H*W][A] f64, moves [i][H*W]
 * (rows past the game's length are zero).  Any output but n_out may be NULL.
 * "Finished" = by the end of the newest move whose games-finished snapshot is
 * complete; if the last enqueued move is still running the drain waits for
 * the move before it, never for the running one (after a synchronizing step
 * or a device synchronize, every finished game). */
int az_selfplay_drain(az_engine* eng, int64_t max_games, int64_t* n_out, int64_t* game_ids,
                      int32_t* lengths, int32_t* results, int32_t* expansions, int8_t* boards,
                      double* policies, int32_t* moves);

/* MCTS tree API (mcts/mcts.py:88-222) over the engine's slots. */
int az_tree_reset(az_engine* eng, int n, const int32_t* slots, const int8_t* boards);
/* Idle the given slots (search and play skip them) until the next reset:
 * an arena's per-move MCTS objects (evaluation/evaluate.py:64-83) use one
 * engine per model and hand each game to the engine whose model moves. */
int az_tree_release(az_engine* eng, int n, const int32_t* slots);
int az_tree_search(az_engine* eng, int n_sims);
/* az_tree_search on an engine created with dirichlet_noise = 1 (ABI 9): the
 * reference draws np.random.dirichlet(alpha * ones(k)) from numpy's global
 * stream at every root selection of MCTS.select (mcts.py:70-85, :113-116),
 * so the caller draws them: noise [slots][rows][A] float64, row r of slot s
 * the normalised vector of its r-th root selection in this search (component
 * i for root edge i; a search on an unexpanded root makes n_sims - 1 root
 * selections, on an expanded one n_sims).  Fails with AZ_E_DEVICE
 * (root-noise-rows-exhausted) when a slot needs more rows. */
int az_tree_search_noise(az_engine* eng, int n_sims, const double* noise, int rows);
/* MCTS.play(greedy, deterministic) (mcts.py:182-222) on every active slot:
 * uniforms [slots] are the np.random.random_sample draws np.random.choice
 * would consume (ignored when deterministic); outputs per slot: moves
 * (action, -1 if the slot was idle), status (0 ongoing / 1 win / 2 draw),
 * policy [slots][A] f64. */
int az_tree_play(az_engine* eng, const double* uniforms, int greedy, int deterministic,
                 int32_t* moves, int32_t* status, double* policy);
/* Tree snapshot of one slot: info = {arena_top, root_first, root_n, ply,
 * game_active}; then the edge arrays (length arena_top). */
int az_tree_info(az_engine* eng, int slot, int64_t* info, float* root_value);
int az_tree_export(az_engine* eng, int slot, double* prior, double* w, int32_t* n, int32_t* child,
                   int32_t* child_n, int32_t* action, float* child_value);

int az_stats_get(az_engine* eng, az_stats* st);
/* plays_inferences reset (self_play.py:145-146: a new best model empties the
 * cache); az_engine_set_weights also clears it. */
int az_cache_clear(az_engine* eng);
/* Bypass (0) or use (1) an allocated cache; results are identical either way. */
int az_cache_enable(az_engine* eng, int on);
/* HIP-event timing for bench.py: on = 1 the conv launches, 2 also the
 * select and expand launches (az_stats conv_* / tree_*), k >= 3 every k-th
 * conv launch of each lane (conv_launches counts the timed ones), 0 off. */
int az_timer_enable(az_engine* eng, int on);
/* The host-built libm pow(k, 0.5) table the kernels use (tests). */
int az_pow_table(az_engine* eng, double* out, int64_t n);

#ifdef __cplusplus
}
#endif

#endif /* AZ_H_ */
