/*
 * az_cpu.c -- native CPU self-play engine: bench.py's cpu_baseline_native
 * line (TEST INFRASTRUCTURE: only bench.py's CPU-baseline leg and tests/ use
 * it; never the product path).
 *
 * SURVEY.md 8(d) asks for a stronger CPU line than the reference's Python
 * (the "C++ az_cpu engine on all cores").  This is the reference's self-play
 * (self_play.py:37-119) with every piece native:
 *   - the MCTS is oracle/az_oracle.c's orc_play_game (bit-exact against the
 *     reference's fixtures, tests/test_oracle.py) with its callback evaluator;
 *   - the evaluator is a batch-1 fp32 C forward of the policy/value network
 *     (model/tensorflow/model.py:152-188; BatchNorm folded on the host,
 *     bench.py fold_for_cpu), 4 pixels x 32 output channels held in registers
 *     per weight stream;
 *   - plays_inferences (mcts.py:122-143, utils.py:38-39) is one insert-only
 *     hash table shared by all threads (the reference shares one Manager
 *     dict between its worker processes);
 *   - one game per thread at a time, T threads (the reference's joblib
 *     fan-out of os.cpu_count() - 1 processes, self_play.py:98-110).
 * Its outputs are not parity-checked bit for bit (fp32 sums in a different
 * order than the GPU); tests/test_cpu_native.py checks the forward against
 * oracle/keras_ref.py and a game against the Python oracle's rules.
 */
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define AZC_F 128
#define AZC_MAX_CELLS 128
#define AZC_MAX_ACTIONS 128
#define AZC_MAX_DEPTH 16

/* from az_oracle.c */
typedef int (*orc_eval_cb)(void* ctx, const int8_t* board, float* probs, float* value);
typedef struct {
    int32_t T, result, status;
    int64_t expansions, terminal_visits, nodes, max_depth;
} orc_game_out;
int orc_play_game(int H, int W, int n, int gravity, int sims, uint32_t seed, int eval_kind, void* table,
                  orc_eval_cb cb, void* cb_ctx, int32_t* moves, uint8_t* greedy, int32_t* n_edges,
                  int32_t* edge_action, double* edge_prior, int64_t* edge_n, double* edge_w, double* policy,
                  int8_t* boards, int64_t* rewards, orc_game_out* out);

/* ------------------------------------------------------------------ network */
/* Folded weights, one flat float array in this order (bench.py fold_for_cpu):
 *   stem  w [9][4][F], b [F]
 *   per block d: conv1 w [9][F][F], b [F]; conv2 w [9][F][F], b [F]; res w [F][F], b [F]
 *   policy conv w [F][2], b [2]; value conv w [F], b [1]
 *   policy dense w [2HW][A], b [A]; value dense1 w [HW][hidden], b [hidden]; dense2 w [hidden], b [1] */
typedef struct {
    int H, W, HW, A, depth, hidden;
    const float *stem_w, *stem_b;
    const float *c1_w[AZC_MAX_DEPTH], *c1_b[AZC_MAX_DEPTH], *c2_w[AZC_MAX_DEPTH], *c2_b[AZC_MAX_DEPTH];
    const float *r_w[AZC_MAX_DEPTH], *r_b[AZC_MAX_DEPTH];
    const float *pc_w, *pc_b, *vc_w, *vc_b, *pd_w, *pd_b, *v1_w, *v1_b, *v2_w, *v2_b;
} azc_net;

int64_t azc_weight_count(int H, int W, int A, int depth, int hidden) {
    const int64_t F = AZC_F, HW = (int64_t)H * W;
    return 9 * 4 * F + F + depth * (2 * (9 * F * F + F) + F * F + F) + 2 * F + 2 + F + 1 + 2 * HW * A + A +
           HW * hidden + hidden + hidden + 1;
}

static float* azc_regroup(const float* w, int cin);
static void net_free(azc_net* n) {
    free((void*)n->stem_w);
    for (int d = 0; d < n->depth; ++d) {
        free((void*)n->c1_w[d]);
        free((void*)n->c2_w[d]);
    }
}

static void net_bind(azc_net* n, const float* w, int H, int W, int A, int depth, int hidden) {
    const int F = AZC_F;
    n->H = H; n->W = W; n->HW = H * W; n->A = A; n->depth = depth; n->hidden = hidden;
    const float* p = w;
#define TAKE(dst, cnt) do { dst = p; p += (cnt); } while (0)
    TAKE(n->stem_w, 9 * 4 * F); TAKE(n->stem_b, F);
    for (int d = 0; d < depth; ++d) {
        TAKE(n->c1_w[d], 9 * F * F); TAKE(n->c1_b[d], F);
        TAKE(n->c2_w[d], 9 * F * F); TAKE(n->c2_b[d], F);
        TAKE(n->r_w[d], F * F); TAKE(n->r_b[d], F);
    }
    /* the 3x3 convs' weights regrouped per 32-channel block (conv3x3) */
    n->stem_w = azc_regroup(n->stem_w, 4);
    for (int d = 0; d < depth; ++d) {
        n->c1_w[d] = azc_regroup(n->c1_w[d], F);
        n->c2_w[d] = azc_regroup(n->c2_w[d], F);
    }
    TAKE(n->pc_w, 2 * F); TAKE(n->pc_b, 2); TAKE(n->vc_w, F); TAKE(n->vc_b, 1);
    TAKE(n->pd_w, 2 * n->HW * A); TAKE(n->pd_b, A);
    TAKE(n->v1_w, n->HW * hidden); TAKE(n->v1_b, hidden); TAKE(n->v2_w, hidden); TAKE(n->v2_b, 1);
#undef TAKE
}

/* out[p][:] = bias + sum over the 3x3 taps and input channels (cin of them) of
 * in[q][ci] * w[tap][ci][:]: blocks of 4 pixels x 32 output channels held in
 * registers (8 vectors of 16 floats) across every (tap, ci); off-board taps
 * read a zero row.  wb is the weight matrix regrouped per 32-channel block,
 * [F/32][9][cin][32] (azc_regroup), so each block streams contiguously. */
typedef float azc_v16 __attribute__((vector_size(64)));
static const float azc_zero_row[AZC_F];
static void conv3x3(const azc_net* n, const float* in, int cin, const float* wb, const float* b, float* out) {
    const int H = n->H, W = n->W, HW = n->HW, F = AZC_F;
    for (int p0 = 0; p0 < HW; p0 += 4) {
        const int np = HW - p0 < 4 ? HW - p0 : 4;
        const float* src[9][4];
        for (int tap = 0; tap < 9; ++tap)
            for (int i = 0; i < 4; ++i) {
                src[tap][i] = azc_zero_row;
                if (i >= np) continue;
                const int p = p0 + i, y = p / W + tap / 3 - 1, x = p % W + tap % 3 - 1;
                if (y >= 0 && y < H && x >= 0 && x < W) src[tap][i] = in + (size_t)(y * W + x) * cin;
            }
        for (int c0 = 0; c0 < F; c0 += 32) {
            azc_v16 a00, a01, a10, a11, a20, a21, a30, a31;
            memcpy(&a00, b + c0, 64);
            memcpy(&a01, b + c0 + 16, 64);
            a10 = a20 = a30 = a00;
            a11 = a21 = a31 = a01;
            const float* wt = wb + (size_t)(c0 / 32) * 9 * cin * 32;
            for (int tap = 0; tap < 9; ++tap, wt += (size_t)cin * 32) {
                const float *s0 = src[tap][0], *s1 = src[tap][1], *s2 = src[tap][2], *s3 = src[tap][3];
                for (int ci = 0; ci < cin; ++ci) {
                    azc_v16 w0, w1;
                    memcpy(&w0, wt + (size_t)ci * 32, 64);
                    memcpy(&w1, wt + (size_t)ci * 32 + 16, 64);
                    const float v0 = s0[ci], v1 = s1[ci], v2 = s2[ci], v3 = s3[ci];
                    a00 += v0 * w0; a01 += v0 * w1;
                    a10 += v1 * w0; a11 += v1 * w1;
                    a20 += v2 * w0; a21 += v2 * w1;
                    a30 += v3 * w0; a31 += v3 * w1;
                }
            }
            float* o = out + (size_t)p0 * F + c0;
            memcpy(o, &a00, 64); memcpy(o + 16, &a01, 64);
            if (np > 1) { memcpy(o + F, &a10, 64); memcpy(o + F + 16, &a11, 64); }
            if (np > 2) { memcpy(o + 2 * F, &a20, 64); memcpy(o + 2 * F + 16, &a21, 64); }
            if (np > 3) { memcpy(o + 3 * F, &a30, 64); memcpy(o + 3 * F + 16, &a31, 64); }
        }
    }
}

/* [9][cin][F] -> [F/32][9][cin][32] */
static float* azc_regroup(const float* w, int cin) {
    const int F = AZC_F;
    float* r = malloc(sizeof(float) * 9 * (size_t)cin * F);
    for (int c0 = 0; c0 < F; c0 += 32)
        for (int tap = 0; tap < 9; ++tap)
            for (int ci = 0; ci < cin; ++ci)
                memcpy(r + (((size_t)(c0 / 32) * 9 + tap) * cin + ci) * 32, w + ((size_t)tap * cin + ci) * F + c0,
                       32 * sizeof(float));
    return r;
}

static void relu(float* x, int n) {
    for (int i = 0; i < n; ++i) x[i] = x[i] > 0.f ? x[i] : 0.f;
}

/* Board.full_state (connect_n/board.py:83-98) of a canonical board, then the
 * network; probs [A], *value */
void azc_forward(const azc_net* n, const int8_t* board, float* probs, float* value) {
    const int HW = n->HW, F = AZC_F, A = n->A;
    float x[AZC_MAX_CELLS * 4];
    static __thread float h[AZC_MAX_CELLS * AZC_F], a[AZC_MAX_CELLS * AZC_F], c[AZC_MAX_CELLS * AZC_F];
    for (int p = 0; p < HW; ++p) {
        x[p * 4 + 0] = board[p] == 0;
        x[p * 4 + 1] = board[p] == 1;
        x[p * 4 + 2] = board[p] == -1;
        x[p * 4 + 3] = 1.f;
    }
    conv3x3(n, x, 4, n->stem_w, n->stem_b, h);
    relu(h, HW * F);
    for (int d = 0; d < n->depth; ++d) {
        conv3x3(n, h, F, n->c1_w[d], n->c1_b[d], a);
        relu(a, HW * F);
        conv3x3(n, a, F, n->c2_w[d], n->c2_b[d], c);
        for (int p = 0; p < HW; ++p) {  /* + BN(conv1x1(h)), ReLU */
            float r[AZC_F];
            memcpy(r, n->r_b[d], sizeof(r));
            const float* hp = h + (size_t)p * F;
            for (int ci = 0; ci < F; ++ci) {
                const float v = hp[ci];
                if (v == 0.f) continue;
                const float* wr = n->r_w[d] + (size_t)ci * F;
                for (int co = 0; co < F; ++co) r[co] += v * wr[co];
            }
            float* cp = c + (size_t)p * F;
            for (int co = 0; co < F; ++co) {
                const float s = cp[co] + r[co];
                cp[co] = s > 0.f ? s : 0.f;
            }
        }
        memcpy(h, c, sizeof(float) * (size_t)HW * F);
    }
    float pf[2 * AZC_MAX_CELLS], vf[AZC_MAX_CELLS];
    for (int p = 0; p < HW; ++p) {
        float s0 = n->pc_b[0], s1 = n->pc_b[1], s2 = n->vc_b[0];
        const float* hp = h + (size_t)p * F;
        for (int ci = 0; ci < F; ++ci) {
            s0 += hp[ci] * n->pc_w[2 * ci];
            s1 += hp[ci] * n->pc_w[2 * ci + 1];
            s2 += hp[ci] * n->vc_w[ci];
        }
        pf[2 * p] = s0 > 0.f ? s0 : 0.f;
        pf[2 * p + 1] = s1 > 0.f ? s1 : 0.f;
        vf[p] = s2 > 0.f ? s2 : 0.f;
    }
    float lg[AZC_MAX_ACTIONS], m = -INFINITY;
    for (int k = 0; k < A; ++k) {
        float s = n->pd_b[k];
        for (int i = 0; i < 2 * HW; ++i) s += pf[i] * n->pd_w[(size_t)i * A + k];
        lg[k] = s;
        m = s > m ? s : m;
    }
    float z = 0.f;
    for (int k = 0; k < A; ++k) {
        lg[k] = expf(lg[k] - m);
        z += lg[k];
    }
    for (int k = 0; k < A; ++k) probs[k] = lg[k] / z;
    float v = n->v2_b[0];
    for (int j = 0; j < n->hidden; ++j) {
        float s = n->v1_b[j];
        for (int p = 0; p < HW; ++p) s += vf[p] * n->v1_w[(size_t)p * n->hidden + j];
        v += (s > 0.f ? s : 0.f) * n->v2_w[j];
    }
    *value = tanhf(v);
}

/* ------------------------------------------------------ shared inference cache */
/* Insert-only open addressing: a slot is claimed by CAS on its state (0 empty,
 * 1 claimed, 2 ready), the key and payload written, then published by a
 * release store; a reader that sees "claimed" evaluates the board itself. */
typedef struct {
    int64_t cap;  /* power of two */
    int A;
    _Atomic uint32_t* state;
    uint64_t* keys;  /* [cap][4] */
    float* pay;      /* [cap][A + 1] */
    atomic_llong hits, inserts, full;
} azc_cache;

static void board_key(const int8_t* b, int HW, uint64_t k[4]) {
    k[0] = k[1] = k[2] = k[3] = 0;
    for (int c = 0; c < HW; ++c) {
        if (b[c] == 1) k[c >> 6] |= 1ull << (c & 63);
        else if (b[c] == -1) k[2 + (c >> 6)] |= 1ull << (c & 63);
    }
}

static uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int cache_get(azc_cache* c, const uint64_t k[4], float* probs, float* value, int64_t* slot_out) {
    const uint64_t h = mix64(mix64(mix64(mix64(k[0]) ^ k[1]) ^ k[2]) ^ k[3]);
    for (int64_t i = 0; i < 64; ++i) {
        const int64_t s = (int64_t)((h + (uint64_t)i) & (uint64_t)(c->cap - 1));
        uint32_t st = atomic_load_explicit(&c->state[s], memory_order_acquire);
        if (st == 0) {
            uint32_t expect = 0;
            if (atomic_compare_exchange_strong(&c->state[s], &expect, 1u)) {
                *slot_out = s;
                return 0;
            }
            st = expect;
        }
        if (st == 2 && memcmp(c->keys + 4 * s, k, 32) == 0) {
            memcpy(probs, c->pay + (size_t)s * (c->A + 1), sizeof(float) * c->A);
            *value = c->pay[(size_t)s * (c->A + 1) + c->A];
            atomic_fetch_add(&c->hits, 1);
            return 1;
        }
        if (st == 1) {
            /* claimed by another thread, maybe this board: evaluate it ourselves */
            *slot_out = -1;
            return 0;
        }
    }
    atomic_fetch_add(&c->full, 1);
    *slot_out = -1;
    return 0;
}

static void cache_put(azc_cache* c, int64_t s, const uint64_t k[4], const float* probs, float value) {
    memcpy(c->keys + 4 * s, k, 32);
    memcpy(c->pay + (size_t)s * (c->A + 1), probs, sizeof(float) * c->A);
    c->pay[(size_t)s * (c->A + 1) + c->A] = value;
    atomic_store_explicit(&c->state[s], 2u, memory_order_release);
    atomic_fetch_add(&c->inserts, 1);
}

/* ------------------------------------------------------------------ self-play */
typedef struct {
    const azc_net* net;
    azc_cache* cache;
    int H, W, n, gravity, sims;
    uint32_t seed0;
    int thread, threads;
    double deadline;
    int64_t games, expansions, evals, plies;
} azc_worker;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int eval_cb(void* ctx, const int8_t* board, float* probs, float* value) {
    azc_worker* w = (azc_worker*)ctx;
    uint64_t k[4];
    board_key(board, w->H * w->W, k);
    int64_t slot = -1;
    if (w->cache && cache_get(w->cache, k, probs, value, &slot)) return 0;
    azc_forward(w->net, board, probs, value);
    w->evals++;
    if (w->cache && slot >= 0) cache_put(w->cache, slot, k, probs, *value);
    return 0;
}

static void* worker_main(void* arg) {
    azc_worker* w = (azc_worker*)arg;
    const int HW = w->H * w->W, A = w->gravity ? w->W : HW;
    int32_t* moves = malloc(sizeof(int32_t) * HW);
    uint8_t* greedy = malloc(HW);
    int32_t* n_edges = malloc(sizeof(int32_t) * HW);
    int32_t* ea = malloc(sizeof(int32_t) * HW * A);
    double* ep = malloc(sizeof(double) * HW * A);
    int64_t* en = malloc(sizeof(int64_t) * HW * A);
    double* ew = malloc(sizeof(double) * HW * A);
    double* pol = malloc(sizeof(double) * HW * A);
    int8_t* boards = malloc((size_t)HW * HW);
    int64_t* rewards = malloc(sizeof(int64_t) * HW);
    /* game k of this thread: seed base + thread + k * threads (distinct games across threads) */
    for (int64_t k = 0; now_s() < w->deadline; ++k) {
        orc_game_out out;
        const uint32_t seed = w->seed0 + (uint32_t)(w->thread + k * w->threads);
        if (orc_play_game(w->H, w->W, w->n, w->gravity, w->sims, seed, 2, NULL, eval_cb, w, moves, greedy,
                          n_edges, ea, ep, en, ew, pol, boards, rewards, &out) != 0)
            break;
        w->games++;
        w->expansions += out.expansions;
        w->plies += out.T;
    }
    free(moves); free(greedy); free(n_edges); free(ea); free(ep); free(en); free(ew); free(pol); free(boards);
    free(rewards);
    return NULL;
}

/* Self-play on `threads` threads for `seconds` (games in progress finish);
 * out[0..5] = games, expansions, network evaluations, plies, cache hits,
 * wall seconds.  cache_log2 = 0: no cache. */
int azc_selfplay(int H, int W, int n, int gravity, int sims, int depth, int hidden, const float* weights,
                 int threads, double seconds, uint32_t seed0, int cache_log2, double* out) {
    const int HW = H * W, A = gravity ? W : HW;
    if (HW > AZC_MAX_CELLS || A > AZC_MAX_ACTIONS || depth > AZC_MAX_DEPTH || threads < 1) return -1;
    azc_net net;
    net_bind(&net, weights, H, W, A, depth, hidden);
    azc_cache cache, *cp = NULL;
    memset(&cache, 0, sizeof(cache));
    if (cache_log2 > 0) {
        cache.cap = (int64_t)1 << cache_log2;
        cache.A = A;
        cache.state = calloc((size_t)cache.cap, sizeof(uint32_t));
        cache.keys = malloc(sizeof(uint64_t) * 4 * (size_t)cache.cap);
        cache.pay = malloc(sizeof(float) * (size_t)(A + 1) * (size_t)cache.cap);
        if (!cache.state || !cache.keys || !cache.pay) return -2;
        cp = &cache;
    }
    azc_worker* ws = calloc((size_t)threads, sizeof(azc_worker));
    pthread_t* th = calloc((size_t)threads, sizeof(pthread_t));
    const double t0 = now_s();
    for (int i = 0; i < threads; ++i) {
        ws[i] = (azc_worker){&net, cp, H, W, n, gravity, sims, seed0, i, threads, t0 + seconds, 0, 0, 0, 0};
        pthread_create(&th[i], NULL, worker_main, &ws[i]);
    }
    for (int i = 0; i < 6; ++i) out[i] = 0.0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        out[0] += (double)ws[i].games;
        out[1] += (double)ws[i].expansions;
        out[2] += (double)ws[i].evals;
        out[3] += (double)ws[i].plies;
    }
    out[4] = cp ? (double)atomic_load(&cache.hits) : 0.0;
    out[5] = now_s() - t0;
    free(ws); free(th);
    net_free(&net);
    if (cp) { free((void*)cache.state); free(cache.keys); free(cache.pay); }
    return 0;
}

/* one forward (tests): board [HW] int8 canonical -> probs [A], value */
int azc_forward_probe(int H, int W, int gravity, int depth, int hidden, const float* weights, const int8_t* board,
                      float* probs, float* value) {
    const int HW = H * W, A = gravity ? W : HW;
    if (HW > AZC_MAX_CELLS || A > AZC_MAX_ACTIONS || depth > AZC_MAX_DEPTH) return -1;
    azc_net net;
    net_bind(&net, weights, H, W, A, depth, hidden);
    azc_forward(&net, board, probs, value);
    net_free(&net);
    return 0;
}
