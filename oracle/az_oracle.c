/*
 * az_oracle.c -- CPU restatement of the reference's Connect-N self-play path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the reported CPU baseline), never as the product path.
 *
 * Parity pinned: tests/test_oracle.py checks every function here against the
 * golden vectors (tests/golden, .npz files), which tests/golden/make_golden.py
 * produced by running the reference itself (numpy 1.26 legacy promotion).
 *
 * What is restated (reference paths relative to /root/reference):
 *   board rules      custom_alphazero/connect_n/board.py:113-124 (moves),
 *                    :154-155 (mask), :178-208 (win/draw), :210-250 (push,
 *                    play with keep_same_player=True -> canonical mirror)
 *   UCB              custom_alphazero/mcts/mcts.py:39-55 (float64 under
 *                    numpy<2 promotion; `** 0.5` is libm pow, not sqrt)
 *   best edge        mcts.py:64-68 (np.argmax -> first maximum)
 *   select           mcts.py:111-120
 *   expand           mcts.py:145-161 + mcts/utils.py:4-16 (float32 pairwise
 *                    sum, float32 divide, float64 uniform on zero sum)
 *   backup           mcts.py:163-168
 *   search           mcts.py:170-180
 *   play             mcts.py:182-222 (np.random.choice: cumsum, normalise by
 *                    the last element, searchsorted 'right' on one legacy
 *                    random_sample = two MT19937 outputs)
 *   play_game        custom_alphazero/self_play.py:37-82 (seeded MT19937,
 *                    greedy from fullmove_number >= 8, alternating rewards)
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, plain SSE2 doubles).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAX_CELLS 128
#define ORC_MAX_ACTIONS 128

typedef struct {
    int H, W, n, gravity, A;
    double c_puct;
    int greedy_ply;
} orc_game;

/* ------------------------------------------------------------ board rules */
/* Board = int8 cells[H*W], row 0 = top (reference `array`), canonical: the
 * side to move owns the +1 stones (board.py:244-246). */

static int orc_action_space(const orc_game* g) { return g->gravity ? g->W : g->W * g->H; }

/* action index -> (x, y) of the stone it places; -1 if illegal. The action
 * order is get_all_possible_moves (board.py:130-146): x for gravity, x-major
 * product(range(W), range(H)) otherwise. */
static int orc_action_cell(const orc_game* g, const int8_t* b, int a) {
    if (g->gravity) {
        int x = a, row = -1;
        for (int y = 0; y < g->H; ++y) {
            if (b[y * g->W + x] != 0) break;
            row = y;
        }
        return row < 0 ? -1 : row * g->W + x;
    }
    int x = a / g->H, y = a % g->H;
    return b[y * g->W + x] == 0 ? y * g->W + x : -1;
}

/* Legal actions in `Board.moves` order (board.py:113-124): ascending column
 * for gravity; np.where row-major (y, then x) without gravity. */
static int orc_moves(const orc_game* g, const int8_t* b, int* out) {
    int k = 0;
    if (g->gravity) {
        for (int x = 0; x < g->W; ++x)
            if (b[x] == 0) out[k++] = x;
    } else {
        for (int y = 0; y < g->H; ++y)
            for (int x = 0; x < g->W; ++x)
                if (b[y * g->W + x] == 0) out[k++] = x * g->H + y;
    }
    return k;
}

/* Legal actions in action (all_possible_moves) order, i.e. legal_moves_mask. */
static int orc_mask_order(const orc_game* g, const int8_t* b, int* out) {
    int k = 0;
    for (int a = 0; a < orc_action_space(g); ++a)
        if (orc_action_cell(g, b, a) >= 0) out[k++] = a;
    return k;
}

/* Play action `a` for the side to move, then mirror (keep_same_player).
 * Returns 0 = ongoing, 1 = the mover connected n (get_result -> 1),
 * 2 = draw (get_result -> 0).  board.py:178-250. */
static int orc_play(const orc_game* g, int8_t* b, int a) {
    static const int dirs[4][2] = {{0, 1}, {1, 1}, {1, 0}, {1, -1}};
    int cell = orc_action_cell(g, b, a);
    if (cell < 0) return -1;
    int x0 = cell % g->W, y0 = cell / g->W;
    b[cell] = 1;
    int status = 0;
    for (int d = 0; d < 4 && !status; ++d) {
        int count = 1;
        for (int sgn = 1; sgn >= -1; sgn -= 2) {
            int dx = dirs[d][0] * sgn, dy = dirs[d][1] * sgn;
            int x = x0 + dx, y = y0 + dy;
            while (x >= 0 && x < g->W && y >= 0 && y < g->H && b[y * g->W + x] == 1) {
                if (++count >= g->n) { status = 1; break; }
                x += dx; y += dy;
            }
            if (status) break;
        }
    }
    if (!status) {
        int tmp[ORC_MAX_ACTIONS];
        if (orc_moves(g, b, tmp) == 0) status = 2;
    }
    for (int i = 0; i < g->H * g->W; ++i) b[i] = (int8_t)-b[i];
    return status;
}

/* ------------------------------------------------------------- numerics */
/* numpy float32 add.reduce (pairwise_sum, PW_BLOCKSIZE 128, 8 accumulators
 * from n >= 8), added to the identity 0. */
static float orc_pairwise_f32(const float* a, long n) {
    if (n < 8) {
        float r = 0.0f;
        for (long i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    return orc_pairwise_f32(a, n2) + orc_pairwise_f32(a + n2, n - n2);
}

static double orc_pairwise_f64(const double* a, long n) {
    if (n < 8) {
        double r = 0.0;
        for (long i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    return orc_pairwise_f64(a, n2) + orc_pairwise_f64(a + n2, n - n2);
}

/* normalize_probabilities on a float32 vector (mcts/utils.py:4-16): returns
 * 1 when the float64 uniform branch was taken. */
int orc_normalize_f32(const float* p, int n, double* out) {
    float s = orc_pairwise_f32(p, n);
    if (s == 0.0f) {
        for (int i = 0; i < n; ++i) out[i] = 1.0 / (double)n;
        return 1;
    }
    for (int i = 0; i < n; ++i) out[i] = (double)(float)(p[i] / s);
    return 0;
}

/* normalize_probabilities on float64 visit counts (mcts.py:194-197). */
void orc_normalize_f64(const double* p, int n, double* out) {
    double s = orc_pairwise_f64(p, n);
    if (s == 0.0) {
        for (int i = 0; i < n; ++i) out[i] = 1.0 / (double)n;
        return;
    }
    for (int i = 0; i < n; ++i) out[i] = p[i] / s;
}

/* Python `int ** 0.5` is float_pow -> libm pow(n, 0.5); 0 ** 0.5 == 0.0.
 * Called through a volatile pointer so no compiler may turn it into sqrt. */
static double (*volatile orc_pow_fn)(double, double) = pow;
double orc_pow_half(int64_t n) { return n == 0 ? 0.0 : orc_pow_fn((double)n, 0.5); }

/* --------------------------------------------------------------- MT19937 */
typedef struct {
    uint32_t mt[624];
    int pos;
} orc_mt;

void orc_mt_seed(orc_mt* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->pos = 624;
}

static uint32_t orc_mt_next(orc_mt* s) {
    if (s->pos >= 624) {
        for (int i = 0; i < 624; ++i) {
            uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
            s->mt[i] = s->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        s->pos = 0;
    }
    uint32_t y = s->mt[s->pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* legacy RandomState.random_sample: 53-bit double from two outputs */
double orc_mt_uniform(orc_mt* s) {
    uint32_t a = orc_mt_next(s) >> 5, b = orc_mt_next(s) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

/* np.random.choice(n, 1, p) given the uniform draw (mtrand choice, replace
 * branch): cdf = cumsum(p); cdf /= cdf[-1]; searchsorted(cdf, u, 'right'). */
int orc_choice(const double* p, int n, double u) {
    double cdf[ORC_MAX_ACTIONS];
    double acc = 0.0;
    for (int i = 0; i < n; ++i) { acc += p[i]; cdf[i] = acc; }
    double last = cdf[n - 1];
    int idx = 0;
    for (int i = 0; i < n; ++i) {
        cdf[i] /= last;
        if (cdf[i] <= u) idx = i + 1;
    }
    return idx;
}

/* ------------------------------------------------ Dirichlet root noise */
/* numpy legacy RandomState.dirichlet (mtrand.pyx) over legacy_standard_gamma
 * (legacy-distributions.c), as np.random.dirichlet runs in the reference
 * (mcts.py:70-85 with ConfigMCTS.enable_dirichlet_noise, config.py:52-54):
 * libm log / pow through volatile pointers, exactly the calls numpy makes. */
static double (*volatile orc_log_fn)(double) = log;

static double orc_std_exponential(orc_mt* s) { return -orc_log_fn(1.0 - orc_mt_uniform(s)); }

/* 0 < shape <= 1 (Johnk / Best rejection of the legacy sampler) */
double orc_legacy_gamma(orc_mt* s, double shape) {
    if (shape == 1.0) return orc_std_exponential(s);
    for (;;) {
        double U = orc_mt_uniform(s);
        double V = orc_std_exponential(s);
        if (U <= 1.0 - shape) {
            double X = orc_pow_fn(U, 1. / shape);
            if (X <= V) return X;
        } else {
            double Y = -orc_log_fn((1 - U) / shape);
            double X = orc_pow_fn(1.0 - shape + shape * Y, 1. / shape);
            if (X <= (V + Y)) return X;
        }
    }
}

/* dirichlet(alpha * ones(k)): gammas, acc, invacc = 1 / acc, d = g * invacc */
void orc_dirichlet(orc_mt* s, double alpha, int k, double* out) {
    double acc = 0.0;
    for (int j = 0; j < k; ++j) {
        out[j] = orc_legacy_gamma(s, alpha);
        acc = acc + out[j];
    }
    double invacc = 1 / acc;
    for (int j = 0; j < k; ++j) out[j] = out[j] * invacc;
}

/* test helper: n draws of dirichlet(alpha * ones(k)) from MT19937(seed) */
void orc_dirichlet_draws(uint32_t seed, double alpha, int k, int n, double* out) {
    orc_mt s;
    orc_mt_seed(&s, seed);
    for (int i = 0; i < n; ++i) orc_dirichlet(&s, alpha, k, out + (size_t)i * k);
}

/* the noise setting of the next orc_play_game calls (ConfigMCTS) */
static int orc_noise_on = 0;
static double orc_noise_alpha = 0.03, orc_noise_ratio = 0.25;
void orc_set_noise(int on, double alpha, double ratio) {
    orc_noise_on = on;
    orc_noise_alpha = alpha;
    orc_noise_ratio = ratio;
}

/* test helpers exposed for the numeric fixtures */
double orc_seed_uniform(uint32_t seed, int k) {
    orc_mt s;
    orc_mt_seed(&s, seed);
    double u = 0.0;
    for (int i = 0; i <= k; ++i) u = orc_mt_uniform(&s);
    return u;
}

/* ------------------------------------------------------------- evaluators */
typedef int (*orc_eval_cb)(void* ctx, const int8_t* board, float* probs, float* value);

#define ORC_M64 0xFFFFFFFFFFFFFFFFull
static uint64_t orc_splitmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void orc_masks(const orc_game* g, const int8_t* b, uint64_t m[4]) {
    m[0] = m[1] = m[2] = m[3] = 0;
    for (int i = 0; i < g->H * g->W; ++i) {
        uint64_t bit = 1ull << (i & 63);
        if (b[i] == 1) m[i >> 6] |= bit;
        else if (b[i] == -1) m[2 + (i >> 6)] |= bit;
    }
}

/* oracle/synth.py:synth_eval, restated in C */
static void orc_synth(const uint64_t m[4], int A, float* probs, float* value) {
    uint64_t h = orc_splitmix(m[0]);
    h = orc_splitmix(h ^ m[1]);
    h = orc_splitmix(h ^ m[2]);
    h = orc_splitmix(h ^ m[3]);
    uint64_t vh = orc_splitmix(h ^ 0x5555555555555555ull);
    *value = (float)(((double)(vh >> 56) - 128.0) / 128.0);
    if ((vh & 0x3F) == 0) {
        for (int a = 0; a < A; ++a) probs[a] = 0.0f;
        return;
    }
    uint64_t w = h;
    for (int a = 0; a < A; ++a) {
        if (a && a % 12 == 0) w = orc_splitmix(w);
        probs[a] = (float)((double)(((w >> (5 * (a % 12))) & 31) + 1) / 64.0);
    }
}

/* Open-addressing table of recorded (board -> probs, value): the replay
 * evaluator that lets the oracle re-run a GPU trajectory with the GPU's own
 * network outputs. */
typedef struct {
    int64_t cap, count, A;
    uint64_t* keys;   /* cap * 4 */
    uint8_t* used;
    float* probs;     /* cap * A */
    float* values;
    int64_t misses;
} orc_table;

static uint64_t orc_key_hash(const uint64_t* k) {
    return orc_splitmix(k[0] ^ orc_splitmix(k[1] ^ orc_splitmix(k[2] ^ orc_splitmix(k[3]))));
}

orc_table* orc_table_new(int64_t n, int64_t A, const uint64_t* keys, const float* probs,
                         const float* values) {
    orc_table* t = (orc_table*)calloc(1, sizeof(orc_table));
    t->cap = 16;
    while (t->cap < 2 * n + 16) t->cap <<= 1;
    t->A = A;
    t->keys = (uint64_t*)calloc((size_t)t->cap * 4, sizeof(uint64_t));
    t->used = (uint8_t*)calloc((size_t)t->cap, 1);
    t->probs = (float*)calloc((size_t)(t->cap * A), sizeof(float));
    t->values = (float*)calloc((size_t)t->cap, sizeof(float));
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t* k = keys + 4 * i;
        uint64_t slot = orc_key_hash(k) & (uint64_t)(t->cap - 1);
        while (t->used[slot] && memcmp(t->keys + 4 * slot, k, 32) != 0)
            slot = (slot + 1) & (uint64_t)(t->cap - 1);
        if (!t->used[slot]) { t->used[slot] = 1; t->count++; }
        memcpy(t->keys + 4 * slot, k, 32);
        memcpy(t->probs + slot * A, probs + i * A, sizeof(float) * (size_t)A);
        t->values[slot] = values[i];
    }
    return t;
}

void orc_table_free(orc_table* t) {
    if (!t) return;
    free(t->keys); free(t->used); free(t->probs); free(t->values); free(t);
}

int64_t orc_table_misses(const orc_table* t) { return t ? t->misses : -1; }

static int orc_table_get(orc_table* t, const uint64_t* k, float* probs, float* value) {
    uint64_t slot = orc_key_hash(k) & (uint64_t)(t->cap - 1);
    while (t->used[slot]) {
        if (memcmp(t->keys + 4 * slot, k, 32) == 0) {
            memcpy(probs, t->probs + slot * t->A, sizeof(float) * (size_t)t->A);
            *value = t->values[slot];
            return 0;
        }
        slot = (slot + 1) & (uint64_t)(t->cap - 1);
    }
    t->misses++;
    return -1;
}

enum { ORC_EVAL_SYNTH = 0, ORC_EVAL_TABLE = 1, ORC_EVAL_CALLBACK = 2 };

typedef struct {
    int kind;
    orc_table* table;
    orc_eval_cb cb;
    void* cb_ctx;
} orc_evaluator;

static int orc_evaluate(const orc_game* g, orc_evaluator* ev, const int8_t* b, float* probs,
                        float* value) {
    if (ev->kind == ORC_EVAL_SYNTH) {
        uint64_t m[4];
        orc_masks(g, b, m);
        orc_synth(m, g->A, probs, value);
        return 0;
    }
    if (ev->kind == ORC_EVAL_TABLE) {
        uint64_t m[4];
        orc_masks(g, b, m);
        return orc_table_get(ev->table, m, probs, value);
    }
    return ev->cb(ev->cb_ctx, b, probs, value);
}

/* ------------------------------------------------------------------- tree */
typedef struct {
    double prior, W;
    int64_t N;
    int child;   /* node index */
    int action;
} orc_edge;

typedef struct {
    int first, count;  /* edges; count == 0 -> leaf */
    int status;        /* 0 ongoing, 1 win for the mover into it, 2 draw */
    int prior64;       /* priors from normalize_probabilities' float64 uniform branch */
} orc_node;

typedef struct {
    orc_game g;
    orc_evaluator ev;
    orc_node* nodes;
    int8_t* boards;
    orc_edge* edges;
    int n_nodes, cap_nodes, n_edges, cap_edges;
    int root;
    int64_t expansions, terminal_visits, max_depth;
    int error;
    orc_mt* rng;  /* the game's np.random stream (root noise draws) */
} orc_tree;

static int orc_new_node(orc_tree* t, const int8_t* board, int status) {
    if (t->n_nodes == t->cap_nodes) {
        t->cap_nodes = t->cap_nodes ? 2 * t->cap_nodes : 1024;
        t->nodes = (orc_node*)realloc(t->nodes, sizeof(orc_node) * (size_t)t->cap_nodes);
        t->boards = (int8_t*)realloc(t->boards, (size_t)t->cap_nodes * (size_t)(t->g.H * t->g.W));
    }
    int id = t->n_nodes++;
    t->nodes[id].first = 0;
    t->nodes[id].count = 0;
    t->nodes[id].status = status;
    t->nodes[id].prior64 = 0;
    memcpy(t->boards + (size_t)id * (size_t)(t->g.H * t->g.W), board, (size_t)(t->g.H * t->g.W));
    return id;
}

static int orc_best_edge(const orc_tree* t, const orc_node* node) {
    const orc_edge* e = t->edges + node->first;
    int64_t sum = 0;
    for (int i = 0; i < node->count; ++i) sum += e[i].N;
    double sq = orc_pow_half(sum);
    int best = 0;
    double best_v = 0.0;
    for (int i = 0; i < node->count; ++i) {
        double q = e[i].N ? e[i].W / (double)e[i].N : 0.0;
        double u = t->g.c_puct * e[i].prior * sq / (double)(1 + e[i].N);
        double ucb = q + u;
        if (i == 0 || ucb > best_v) { best = i; best_v = ucb; }
    }
    return best;
}

/* get_best_edge_with_noise (mcts.py:70-85): priors as the reference holds
 * them (a float32 array, or float64 from the uniform branch), noisy =
 * (1 - ratio) * priors (in the priors' dtype, numpy legacy promotion) +
 * ratio * dirichlet (float64), UCB with the noisy prior, np.argmax (first
 * maximum; a NaN counts as the maximum, the first NaN wins). */
static int orc_best_edge_noise(orc_tree* t, const orc_node* node) {
    const orc_edge* e = t->edges + node->first;
    double d[ORC_MAX_ACTIONS];
    orc_dirichlet(t->rng, orc_noise_alpha, node->count, d);
    int64_t sum = 0;
    for (int i = 0; i < node->count; ++i) sum += e[i].N;
    double sq = orc_pow_half(sum);
    int best = 0;
    double best_v = 0.0;
    for (int i = 0; i < node->count; ++i) {
        double kept = node->prior64 ? (1 - orc_noise_ratio) * e[i].prior
                                    : (double)((float)(1 - orc_noise_ratio) * (float)e[i].prior);
        double noisy = kept + orc_noise_ratio * d[i];
        double q = e[i].N ? e[i].W / (double)e[i].N : 0.0;
        double u = t->g.c_puct * noisy * sq / (double)(1 + e[i].N);
        double ucb = q + u;
        if (i == 0) { best = 0; best_v = ucb; continue; }
        if (best_v != best_v) continue;                       /* a NaN already holds the max */
        if (ucb != ucb || ucb > best_v) { best = i; best_v = ucb; }
    }
    return best;
}

/* evaluate_and_expand: returns the leaf's value (side to move at the leaf) */
static double orc_expand(orc_tree* t, int node_id) {
    const orc_game* g = &t->g;
    float probs[ORC_MAX_ACTIONS], value = 0.0f;
    int8_t* board = t->boards + (size_t)node_id * (size_t)(g->H * g->W);
    if (orc_evaluate(g, &t->ev, board, probs, &value) != 0) t->error = 1;
    int legal[ORC_MAX_ACTIONS], moves[ORC_MAX_ACTIONS];
    float masked[ORC_MAX_ACTIONS];
    double priors[ORC_MAX_ACTIONS];
    int nl = orc_mask_order(g, board, legal);
    for (int i = 0; i < nl; ++i) masked[i] = probs[legal[i]];
    const int prior64 = orc_normalize_f32(masked, nl, priors);
    int nm = orc_moves(g, board, moves);
    if (t->n_edges + nm > t->cap_edges) {
        while (t->n_edges + nm > t->cap_edges) t->cap_edges = t->cap_edges ? 2 * t->cap_edges : 4096;
        t->edges = (orc_edge*)realloc(t->edges, sizeof(orc_edge) * (size_t)t->cap_edges);
    }
    int first = t->n_edges;
    for (int i = 0; i < nm; ++i) {
        int8_t child_board[ORC_MAX_CELLS];
        memcpy(child_board, t->boards + (size_t)node_id * (size_t)(g->H * g->W), (size_t)(g->H * g->W));
        int status = orc_play(g, child_board, moves[i]);
        int child = orc_new_node(t, child_board, status);
        orc_edge* e = t->edges + first + i;
        e->prior = priors[i];  /* zip(probabilities, moves): positional */
        e->W = 0.0;
        e->N = 0;
        e->child = child;
        e->action = moves[i];
    }
    t->n_edges += nm;
    t->nodes[node_id].first = first;  /* node pointer may have moved */
    t->nodes[node_id].count = nm;
    t->nodes[node_id].prior64 = prior64;
    t->expansions++;
    return (double)value;
}

static void orc_search(orc_tree* t, int sims) {
    int path[ORC_MAX_CELLS + 2];
    for (int s = 0; s < sims; ++s) {
        int depth = 0, node = t->root;
        while (t->nodes[node].count) {
            /* select (mcts.py:111-120): the noisy choice at the current root */
            int k = orc_noise_on && node == t->root ? orc_best_edge_noise(t, t->nodes + node)
                                                    : orc_best_edge(t, t->nodes + node);
            int e = t->nodes[node].first + k;
            path[depth++] = e;
            node = t->edges[e].child;
        }
        if (depth > t->max_depth) t->max_depth = depth;
        double v;
        if (t->nodes[node].status == 0) {
            v = -orc_expand(t, node);
        } else {
            v = t->nodes[node].status == 1 ? 1.0 : 0.0;
            t->terminal_visits++;
        }
        for (int i = depth - 1; i >= 0; --i) {
            t->edges[path[i]].N += 1;
            t->edges[path[i]].W += v;
            v = -v;
        }
    }
}

/* ------------------------------------------------------------- play_game */
typedef struct {
    int32_t T, result, status;
    int64_t expansions, terminal_visits, nodes, max_depth;
} orc_game_out;

/*
 * One self-play game (self_play.py:37-82) from the empty board.
 * Output arrays are sized for T_max = H*W plies:
 *   moves[T], greedy[T], n_edges[T], edge_action/prior/n/w[T][A] (root edges
 *   at the moment each move was played), policy[T][A] (float64), boards[T][H*W]
 *   (the canonical root board before each move), rewards[T] (int64).
 */
/* MT19937 words each game's stream discards after seeding; -1 = the
 * reference play_game's model-construction draws, 2 * H * W * 4 */
static int orc_rng_skip = -1;
void orc_set_rng_skip(int words) { orc_rng_skip = words; }

int orc_play_game(int H, int W, int n, int gravity, int sims, uint32_t seed, int eval_kind,
                  orc_table* table, orc_eval_cb cb, void* cb_ctx, int32_t* moves, uint8_t* greedy,
                  int32_t* n_edges, int32_t* edge_action, double* edge_prior, int64_t* edge_n,
                  double* edge_w, double* policy, int8_t* boards, int64_t* rewards,
                  orc_game_out* out) {
    orc_tree t;
    memset(&t, 0, sizeof(t));
    t.g.H = H; t.g.W = W; t.g.n = n; t.g.gravity = gravity;
    t.g.A = orc_action_space(&t.g);
    t.g.c_puct = 1.5;
    t.g.greedy_ply = 8;
    t.ev.kind = eval_kind;
    t.ev.table = table;
    t.ev.cb = cb;
    t.ev.cb_ctx = cb_ctx;
    const int A = t.g.A, HW = H * W;
    if (HW > ORC_MAX_CELLS || A > ORC_MAX_ACTIONS) return -1;
    orc_mt rng;
    orc_mt_seed(&rng, seed);
    /* self_play.play_game seeds np.random, then builds the model, whose
     * constructor runs a dummy forward on np.random.rand(1, H, W, 4)
     * (model/tensorflow/model.py:167-169): 2 words per double */
    const int skip = orc_rng_skip >= 0 ? orc_rng_skip : 2 * HW * 4;
    for (int i = 0; i < skip; ++i) (void)orc_mt_next(&rng);
    t.rng = &rng;
    int8_t board[ORC_MAX_CELLS];
    memset(board, 0, sizeof(board));
    t.root = orc_new_node(&t, board, 0);
    int status = 0, T = 0;
    while (status == 0) {
        orc_search(&t, sims);
        orc_node* root = t.nodes + t.root;
        orc_edge* e = t.edges + root->first;
        int ne = root->count;
        int is_greedy = T >= t.g.greedy_ply;
        double probs[ORC_MAX_ACTIONS];
        if (is_greedy) {
            int best = 0;
            for (int i = 1; i < ne; ++i)
                if (e[i].N > e[best].N) best = i;
            for (int i = 0; i < ne; ++i) probs[i] = i == best ? 1.0 : 0.0;
        } else {
            double counts[ORC_MAX_ACTIONS];
            for (int i = 0; i < ne; ++i) counts[i] = (double)e[i].N;
            orc_normalize_f64(counts, ne, probs);
        }
        double u = orc_mt_uniform(&rng);
        int k = orc_choice(probs, ne, u);
        memcpy(boards + (size_t)T * HW, board, (size_t)HW);
        moves[T] = e[k].action;
        greedy[T] = (uint8_t)is_greedy;
        n_edges[T] = ne;
        for (int i = 0; i < A; ++i) {
            edge_action[(size_t)T * A + i] = i < ne ? e[i].action : -1;
            edge_prior[(size_t)T * A + i] = i < ne ? e[i].prior : 0.0;
            edge_n[(size_t)T * A + i] = i < ne ? e[i].N : 0;
            edge_w[(size_t)T * A + i] = i < ne ? e[i].W : 0.0;
            policy[(size_t)T * A + i] = 0.0;
        }
        for (int i = 0; i < ne; ++i) policy[(size_t)T * A + e[i].action] = probs[i];
        status = orc_play(&t.g, board, e[k].action);
        t.root = e[k].child;
        T++;
    }
    int result = status == 1 ? 1 : 0;
    for (int i = 0; i < T; ++i) rewards[i] = result;
    for (int i = T - 2; i >= 0; i -= 2) rewards[i] = -rewards[i];
    out->T = T;
    out->result = result;
    out->status = t.error ? -2 : 0;
    out->expansions = t.expansions;
    out->terminal_visits = t.terminal_visits;
    out->nodes = t.n_nodes;
    out->max_depth = t.max_depth;
    free(t.nodes); free(t.boards); free(t.edges);
    return t.error ? -2 : 0;
}

/* board-rule probe for the fixtures: plays `n_moves` actions from the empty
 * board, recording the canonical board and status after each. */
int orc_board_replay(int H, int W, int n, int gravity, const int32_t* actions, int n_moves,
                     int8_t* boards_out, int32_t* status_out, uint8_t* mask_out, int32_t* moves_out) {
    orc_game g = {H, W, n, gravity, 0, 1.5, 8};
    g.A = orc_action_space(&g);
    int8_t b[ORC_MAX_CELLS];
    memset(b, 0, sizeof(b));
    for (int i = 0; i < n_moves; ++i) {
        int s = orc_play(&g, b, actions[i]);
        if (s < 0) return -1;
        status_out[i] = s;
        memcpy(boards_out + (size_t)i * H * W, b, (size_t)(H * W));
        for (int a = 0; a < g.A; ++a) mask_out[(size_t)i * g.A + a] = orc_action_cell(&g, b, a) >= 0;
        int mv[ORC_MAX_ACTIONS];
        int k = orc_moves(&g, b, mv);
        for (int a = 0; a < g.A; ++a) moves_out[(size_t)i * g.A + a] = a < k ? mv[a] : -1;
    }
    return 0;
}

/* synthetic evaluator probe (checks the C restatement of oracle/synth.py) */
void orc_synth_probe(int H, int W, int gravity, const int8_t* board, float* probs, float* value) {
    orc_game g = {H, W, 4, gravity, 0, 1.5, 8};
    g.A = orc_action_space(&g);
    uint64_t m[4];
    orc_masks(&g, board, m);
    orc_synth(m, g.A, probs, value);
}
