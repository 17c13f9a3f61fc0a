/*
 * az_chess.h -- C ABI of libaz's chess board kernels (gfx950).
 *
 * Replaces the reference's chess board seam (custom_alphazero/chess/), which
 * is a subclass of python-chess 1.9.4 (poetry.lock:227-228): the hot path's
 * "board-tensor encode + legal-move mask" for chess.
 * Each call below is batched over n positions and runs on the GPU; the Python
 * drop-in (custom_alphazero/chess/board.py) binds them with ctypes.
 *
 * Conventions as in az.h: 0 or a negative AZ_E* code, az_last_error() holds
 * the message; host buffers owned by the caller; synchronous.  `device` is a
 * HIP device ordinal; each call uses a per-device stream and scratch of the
 * library's own.
 *
 * Squares are python-chess's (A1 = 0 .. H8 = 63).  A move is a uint16:
 * from | to << 6 | promotion << 12, promotion = python-chess piece type
 * (0 none, 2 knight, 3 bishop, 4 rook, 5 queen).
 */
#ifndef AZ_CHESS_H_
#define AZ_CHESS_H_

#include <stdint.h>

#include "az.h"

#ifdef __cplusplus
extern "C" {
#endif

#define AZ_CHESS_MAX_MOVES 256  /* > 218, the most legal moves of any position */
#define AZ_CHESS_ACTIONS 1880   /* len(get_all_possible_moves()) (chess/utils.py:11-32) */
#define AZ_CHESS_HISTORY 8      /* Board(history_size=8) (chess/board.py:17) */
#define AZ_CHESS_PLANES 118     /* 8 x (13 one-hot + repetition) + 6 (chess/board.py:55-73) */

/* A python-chess Board's position state (80 bytes).  The repetition flag is
 * the value Board.state's last plane carries (is_repetition()). */
typedef struct az_chess_pos {
    uint64_t pieces[6];        /* pawns, knights, bishops, rooks, queens, kings */
    uint64_t occupied_co[2];   /* [0] BLACK, [1] WHITE */
    uint64_t castling_rights;  /* rook squares (python-chess Board.castling_rights) */
    int16_t ep_square;         /* -1 = None */
    uint8_t turn;              /* 1 = WHITE */
    uint8_t repetition;
    uint16_t halfmove_clock;
    uint16_t fullmove_number;
} az_chess_pos;

/* Termination codes of python-chess Board.outcome() (checked in this order) */
#define AZ_CHESS_ONGOING 0
#define AZ_CHESS_CHECKMATE 1
#define AZ_CHESS_INSUFFICIENT 2
#define AZ_CHESS_STALEMATE 3
#define AZ_CHESS_SEVENTYFIVE 4

/* get_all_possible_moves() (chess/utils.py:11-32): the action list, sorted by
 * Move.__lt__ (chess/move.py:33-37).  cap >= AZ_CHESS_ACTIONS; returns the
 * count (host-side table, no device work). */
int az_chess_all_moves(uint16_t* out, int cap);

/* Board.moves (chess/board.py:46-48: python-chess legal_moves, generation
 * order), Board.legal_moves_mask(all_possible_moves) (:111-112) and
 * is_game_over()/outcome() for n positions: moves [n][AZ_CHESS_MAX_MOVES],
 * counts [n], mask [n][AZ_CHESS_ACTIONS] u8, outcome [n].  Any output except
 * counts may be NULL. */
int az_chess_legal(int device, const az_chess_pos* pos, int n, uint16_t* moves, int32_t* counts,
                   uint8_t* mask, int32_t* outcome);

/* Board.full_state (chess/board.py:55-73) for n boards: hist [n][8] oldest
 * first (the state_history deque), valid [n][8] (0 = a zero-filled entry),
 * the board itself is hist[i][7] (castling planes, fullmove, halfmove) ->
 * state [n][8][8][118] f32, rows = ranks 8..1 as Board.array (every value is
 * a small integer: exact in f32; the reference's float64 casts exactly). */
int az_chess_encode(int device, const az_chess_pos* hist, const uint8_t* valid, int n,
                    float* state);

/* Board.play(move, keep_same_player=...) (chess/board.py:162-173) in place on
 * n positions: push, then (keep_same_player) mirror + turn = WHITE. */
int az_chess_play(int device, az_chess_pos* pos, const uint16_t* moves, int n,
                  int keep_same_player);

/* perft(depth) node count (legal move generation + push, breadth first on the
 * device): the size-independent check of the move generator. */
int az_chess_perft(int device, const az_chess_pos* pos, int depth, uint64_t* nodes);


/* ------------------------------------------------------------ self-play
 * Chess self-play (BASELINE configs[4]): the batched
 * replacement of self_play.play_game / MCTS on chess boards
 * (self_play.py:37-82, mcts/mcts.py:88-222, chess/board.py).  Same tree
 * arithmetic as the Connect-N engine (f64 PUCT, libm pow, first-max argmax,
 * float32 pairwise prior normalisation with the reference's positional
 * prior/move zip, np.random.choice on MT19937); subtrees are reused across
 * moves (current_root = edge.child) and compacted into the other half of the
 * slot's edge arena.  The reference's chess path cannot finish a game under
 * MCTS (get_result() takes no keep_same_player, chess/board.py:178 vs
 * mcts.py:179); here a terminal board scores as get_result does in the
 * canonical form: 1 for checkmate (a win for the side that just moved), 0 for
 * every draw. */
typedef struct az_chess_engine az_chess_engine;

typedef struct az_chess_config {
    int32_t mcts_iterations;      /* sims per move (ConfigSelfPlay.mcts_iterations) */
    int32_t index_move_greedy;    /* greedy once fullmove_number >= this (self_play.py:62) */
    double exploration_constant;  /* ConfigMCTS.exploration_constant */
    int32_t slots;                /* concurrent games on this device */
    int32_t evaluator;            /* AZ_EVAL_NETWORK or AZ_EVAL_SYNTHETIC */
    int32_t filters, depth, value_hidden;  /* ConfigModel (filters must be 128) */
    int32_t max_plies;            /* addition: games stop (as draws) after this many plies;
                                     the reference has no cap (0 = 512) */
    double bn_epsilon;
    int64_t arena_edges;          /* edges per arena half per slot (0 = 96 * mcts_iterations) */
    int32_t conv_algo;            /* AZ_CONV_F16X2 (default) / AZ_CONV_DIRECT: the tower and the
                                     stem over the 118 planes zero-padded to 128 */
    int32_t lanes;                /* slot groups searched on separate HIP streams (0 = auto: 2 from
                                     128 slots, else 1); results do not depend on it */
    int32_t cache_log2;           /* ABI 10: transposition cache entries = 2^cache_log2, the
                                     reference's plays_inferences on chess boards (mcts.py:122-143):
                                     key = the leaf position + its history form, ~1.1 KB per entry
                                     (the masked priors, up to 256, and the value); identical leaves
                                     of one simulation share a network row.  0 = off, else 4..28;
                                     results are identical either way */
    int32_t reserved[5];
} az_chess_config;
/* Scope: no Dirichlet root noise (ConfigMCTS.enable_dirichlet_noise,
 * mcts.py:70-85) in the chess engine.  The reference's chess MCTS cannot run
 * a search at all (chess/board.py:178's get_result signature vs mcts.py:179),
 * so there is no noisy chess behaviour to match; the Python layer refuses
 * the flag for chess (config.check_mcts_config("chess")) instead of
 * ignoring it.  Connect-N has it in self-play and in the tree API (az.h). */

/* Termination of a finished self-play game: AZ_CHESS_* above, or this */
#define AZ_CHESS_MAX_PLIES 5

int az_chess_engine_create(int device, const az_chess_config* cfg, az_chess_engine** out);
int az_chess_engine_destroy(az_chess_engine* eng);
/* PolicyValueModel weights for input_dim (8, 8, 118), action_space 1880
 * (model/tensorflow/model.py:152-188; names of custom_alphazero/model/weights.py) */
int az_chess_engine_set_weights(az_chess_engine* eng, const az_tensor* tensors, int n);
/* PolicyValueModel.__call__ on chess states: x [n][8][8][118] f32 (Board.full_state)
 * -> probs [n][1880] f32, values [n] f32 */
int az_chess_forward(az_chess_engine* eng, const float* x, int n, float* probs, float* values);
/* Games first_game .. first_game + n_games - 1 from the start position, game g
 * seeded with MT19937(base_seed + g); slots refilled as games end. */
int az_chess_selfplay_begin(az_chess_engine* eng, int64_t first_game, int64_t n_games,
                            uint32_t base_seed);
/* With st = NULL the moves are only enqueued (ABI 10): the call returns at once
 * and device errors surface at the next synchronizing call; with st it waits
 * for them and fills the stats. */
int az_chess_selfplay_step(az_chess_engine* eng, int n_moves, az_stats* st);
int az_chess_selfplay_run(az_chess_engine* eng, int64_t first_game, int64_t n_games,
                          uint32_t base_seed, az_stats* st);
/* Per game g (P = max_plies): lengths[g] plies; results[g] (1 checkmate, 0
 * draw or cap); terminations[g] (AZ_CHESS_*); expansions[g]; positions
 * [g][P] (canonical root before each move, MCTS.play's parent board); moves
 * [g][P]; the MCTS.play policy sparsely: policy_n [g][P] root edges,
 * policy_actions [g][P][AZ_CHESS_MAX_MOVES] action indices (edge order),
 * policy_probs [g][P][AZ_CHESS_MAX_MOVES] f64.  Any pointer may be NULL. */
int az_chess_selfplay_results(az_chess_engine* eng, int32_t* lengths, int32_t* results,
                              int32_t* terminations, int32_t* expansions, az_chess_pos* positions,
                              uint16_t* moves, int32_t* policy_n, int16_t* policy_actions,
                              double* policy_probs);
/* The games that finished since the previous drain (ABI 10; at most
 * max_games, in the order they finished) while self-play runs on: the
 * reference's result return (self_play.py:112-118), one step at a time, as
 * az_selfplay_drain does for Connect-N.  *n_out = games copied; per game i:
 * game_ids[i], lengths/results/terminations/expansions[i], and its rows as
 * az_chess_selfplay_results: positions [i][P], moves [i][P], policy_n
 * [i][P], policy_actions [i][P][AZ_CHESS_MAX_MOVES], policy_probs
 * [i][P][AZ_CHESS_MAX_MOVES] (P = max_plies; rows past the game's length are
 * zero).  "Finished" = by the end of the newest move whose games-finished
 * snapshot is complete: the drain never waits for a running move.  Any
 * output but n_out may be NULL. */
int az_chess_selfplay_drain(az_chess_engine* eng, int64_t max_games, int64_t* n_out, int64_t* game_ids,
                            int32_t* lengths, int32_t* results, int32_t* terminations, int32_t* expansions,
                            az_chess_pos* positions, uint16_t* moves, int32_t* policy_n,
                            int16_t* policy_actions, double* policy_probs);
int az_chess_stats(az_chess_engine* eng, az_stats* st);

/* MCTS tree API on chess boards (mcts/mcts.py:86-222 with a chess Board):
 * replaces the per-object UCTNode/UCTEdge tree of one MCTS instance with a
 * slot of the engine.  A reset root evaluates with the history of a board
 * made by deepcopy (python-chess copy() re-runs the subclass __init__:
 * [0 x 7, start-position state], whatever the position); every board after
 * play() holds [0 x 6, start state, board].  Positions are canonical
 * (Board.play(keep_same_player=True) form). */
int az_chess_tree_reset(az_chess_engine* eng, int n, const int32_t* slots, const az_chess_pos* roots);
/* Idle the given slots (search and play skip them) until the next reset. */
int az_chess_tree_release(az_chess_engine* eng, int n, const int32_t* slots);
/* MCTS.search(n_sims) on every active slot. */
int az_chess_tree_search(az_chess_engine* eng, int n_sims);
/* MCTS.play(greedy, deterministic) on every active slot: uniforms [slots] are
 * the np.random.random_sample draws np.random.choice consumes (ignored when
 * deterministic).  Per slot: moves (move code, -1 idle), status (AZ_CHESS_*
 * outcome of the new root), the policy sparsely as in
 * az_chess_selfplay_results (policy_n, policy_actions [slots][256], policy_probs
 * [slots][256]).  The chosen child's subtree becomes the tree (mcts.py:212);
 * siblings are dropped.  Any output pointer may be NULL. */
int az_chess_tree_play(az_chess_engine* eng, const double* uniforms, int greedy, int deterministic,
                       int32_t* moves, int32_t* status, int32_t* policy_n, int16_t* policy_actions,
                       double* policy_probs);
/* Tree snapshot of one slot: info = {edges, root_first, root_n, ply,
 * active}, root_value = the root's evaluated_value (0 before expansion);
 * then the edge arrays (length info[0]); moves are move codes, child the
 * first edge of the child's expansion or -1. */
int az_chess_tree_info(az_chess_engine* eng, int slot, int64_t* info, float* root_value);
int az_chess_tree_export(az_chess_engine* eng, int slot, double* prior, double* w, int32_t* n,
                         int32_t* child, int32_t* child_n, int32_t* moves, float* child_value);

/* HIP-event timing of the residual-tower conv launches (bench.py roofline) */
int az_chess_timer_enable(az_chess_engine* eng, int on);

#ifdef __cplusplus
}
#endif
#endif
