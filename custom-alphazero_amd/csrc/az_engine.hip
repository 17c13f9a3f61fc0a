// az_engine.hip -- host side of libaz: the C ABI (include/az.h), device
// buffers, BatchNorm folding, and the lockstep self-play driver.
#include <math.h>
#include <string.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "../../include/az.h"
#include "az_nn.h"
#include "az_tree.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define AZ_HIP(expr)                                                                    \
  do {                                                                                  \
    hipError_t err__ = (expr);                                                          \
    if (err__ != hipSuccess)                                                            \
      return fail(AZ_E_HIP, std::string(#expr) + ": " + hipGetErrorString(err__));      \
  } while (0)

// libm pow through a volatile pointer: Python's `int ** 0.5` (mcts.py:50) is
// float_pow -> pow(n, 0.5), which is NOT sqrt for 1,638 n <= 2e6.
double (*volatile g_pow)(double, double) = pow;

// HIP hardware queues of this process (GPU_MAX_HW_QUEUES, HIP's default 4),
// read once when the library loads -- HIP reads the variable at its own
// initialisation, so a value set later would not describe the queues HIP
// made; the lane rule (az_engine_lanes) uses this snapshot.  The Python
// package sets 8 at import before anything initialises HIP.
int read_hw_queues() {
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  const int v = q && *q ? atoi(q) : 0;
  return v > 0 ? v : 4;
}
const int g_hw_queues_at_load = read_hw_queues();

}  // namespace

namespace az {
// error reporting for the other ABI translation units (az_chess.hip)
int fail_abi(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace az

// A lane = a contiguous group of slots searched on its own HIP stream.  Lanes
// share the network, the transposition cache, the sample sink and the
// counters; each owns its eval queue, per-simulation dedup table and slices
// of the activation buffers.  Two lanes keep the GPU busy across each
// other's launch tails and small latency-bound kernels; results do not
// depend on the lane count (each game's search only reads its own tree and
// the evaluator is deterministic per board).
struct Lane {
  int first = 0, n = 0;
  int32_t* counts = nullptr;  // [2][4][kCountStride] eval/miss/nn/dup counts by simulation parity
  hipStream_t stream = nullptr;
  az::GameCfg g{};
  az::TreeDev t{};
  float* x = nullptr;
  float* act[3] = {nullptr, nullptr, nullptr};
  float* probs = nullptr;
  float* values = nullptr;
  az::ConvTimer timer;
  az::ConvTimer tree_timer;  // select and expand launches (bench.py roofline_tree)
  hipEvent_t move_done[4] = {nullptr, nullptr, nullptr, nullptr};  // end of move m on this lane, m mod 4
  int64_t pool_cap = 0;        // compacted self-play: edges per pool half (TreeDev::pool_cap)
};

struct az_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  Lane whole;                // every slot on `stream` (tree API; self-play with one lane)
  std::vector<Lane*> lanes;  // self-play lanes (just &whole when there is one)
  az_config cfg{};
  az::GameCfg g{};
  az::TreeDev t{};
  az::SampleDev smp{};
  az::CacheDev cache{};
  az::NetDev net{};
  az::ConvTimer timer;
  float* x = nullptr;
  float* act[3] = {nullptr, nullptr, nullptr};
  float* probs = nullptr;
  float* values = nullptr;
  // AZ_EVAL_HOST: the callback and its pinned staging buffers (slots leaves)
  az_eval_fn host_fn = nullptr;
  void* host_user = nullptr;
  float* host_x = nullptr;
  float* host_p = nullptr;
  float* host_v = nullptr;
  int32_t* host_n = nullptr;
  double* uniforms = nullptr;
  double* noise_buf = nullptr;  // az_tree_search_noise: the caller's root-noise rows
  size_t noise_cap = 0;
  int32_t* dev_i32 = nullptr;  // scratch for az_tree_reset
  az::Board* dev_boards = nullptr;
  std::vector<void*> owned;
  std::vector<void*> sample_bufs;
  std::vector<hipStream_t> lane_streams;
  hipEvent_t timer_ref = nullptr;  // common origin of every ConvTimer's intervals
  int64_t sp_first = 0, sp_n = 0;
  int64_t moves_issued = 0;        // self-play moves enqueued (lane drift bound, az_tree.h)
  uint32_t leaf_epoch = 0;         // simulations enqueued, every lane's (TreeDev::leaf_epoch)
  int64_t drained = 0;             // finished games az_selfplay_drain has returned
  uint8_t* drain_dev = nullptr;    // packed records (device) and their pinned host copy
  uint8_t* drain_host = nullptr;
  // games-finished count at the end of every move: the last lane to finish
  // move m stores smp.done_count into snap_host[m % 4] (move_end_kernel), and
  // the drain packs up to a completed snapshot on pack_stream, so it never
  // waits for the move that is running (az_selfplay_step without stats returns
  // without a sync).  No stream of its own: HIP maps streams onto 4 hardware
  // queues per process (GPU_MAX_HW_QUEUES), and a snapshot or pack stream
  // sharing a lane's queue runs behind that lane's queued moves -- with two
  // lanes the pack uses `stream`, idle while moves run.
  hipStream_t pack_stream = nullptr;
  bool own_pack_stream = false;
  int32_t* move_arrive = nullptr;           // [4] lanes done with move m, slot m % 4
  unsigned long long* snap_host = nullptr;  // [4] pinned coherent, move m in slot m % 4
  unsigned long long* snap_dev = nullptr;   // snap_host's device address
  int64_t batch_first_move = 0;             // moves_issued at az_selfplay_begin
  size_t drain_cap = 0;            // records the two buffers hold
  // a host evaluator failed mid-simulation (AZ_E_CALLBACK): the leaves it
  // selected were never expanded, so the trees are one simulation short;
  // searching refuses until az_selfplay_begin or az_tree_reset starts over
  bool broken = false;

  template <typename T>
  int alloc(T** p, size_t count) {
    void* q = nullptr;
    AZ_HIP(hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)));
    owned.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return 0;
  }
};

namespace {

int check_device_errors(az_engine* e) {
  unsigned long long err = 0;
  AZ_HIP(hipMemcpy(&err, e->t.stats + az::kStatErrors, sizeof(err), hipMemcpyDeviceToHost));
  if (err) {
    std::string m = "device error flags:";
    if (err & az::kErrArena) m += " arena-overflow(raise az_config.arena_edges)";
    if (err & az::kErrPow) m += " visit-table-overflow(raise az_config.max_tree_visits)";
    if (err & az::kErrPath) m += " path-overflow";
    if (err & az::kErrIllegal) m += " illegal-move";
    if (err & az::kErrNoRoot) m += " play-before-search";
    if (err & az::kErrNoise) m += " root-noise-rows-exhausted(pass a row per root selection)";
    if (err & az::kErrActRange)
      m += " activation-range(a non-finite activation, or |x| > 32752 in the per-layer fp16x2 convs: "
           "use conv_algo=AZ_CONV_F16X2 or AZ_CONV_DIRECT)";
    // play on a slot without a searched root changes nothing: that flag is
    // cleared once reported (the others mean a broken tree and stay)
    if (err == az::kErrNoRoot) AZ_HIP(hipMemset(e->t.stats + az::kStatErrors, 0, sizeof(err)));
    return fail(AZ_E_DEVICE, m);
  }
  return 0;
}

az::Board board_from_cells(const int8_t* cells, int HW) {
  az::Board b;
  b.own[0] = b.own[1] = b.opp[0] = b.opp[1] = 0;
  for (int c = 0; c < HW; ++c) {
    if (cells[c] == 1) az::set_bit(b.own, c);
    else if (cells[c] == -1) az::set_bit(b.opp, c);
  }
  return b;
}

// point a tree view's four counters at parity p of the [2][4] block at base
void set_counts(az::TreeDev& t, int32_t* base, int p) {
  constexpr int K = az::kCountStride;
  t.eval_count = base + 4 * K * p;
  t.miss_count = t.eval_count + K;
  t.nn_count = t.eval_count + 2 * K;
  t.next_counts = base + 4 * K * (p ^ 1);
}

void cells_from_board(const az::Board& b, int HW, int8_t* cells) {
  for (int c = 0; c < HW; ++c)
    cells[c] = az::bit(b.own, c) ? 1 : (az::bit(b.opp, c) ? -1 : 0);
}

// AZ_EVAL_HOST: the leaves' full_state planes to the host, the callback (the
// reference's self.model(np.expand_dims(board.full_state, 0)), mcts.py:130-137,
// here over every leaf of the simulation at once), its outputs back to the
// lane's evaluator slices; synchronous on the lane's stream
int host_evaluate(az_engine* e, Lane& L, const az::Board* rows, const int32_t* n_rows) {
  hipStream_t s = L.stream;
  const int HW = L.g.HW, A = L.g.A;
  az::launch_encode(rows, n_rows, L.n, HW, L.x, s);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipMemcpyAsync(e->host_n, n_rows, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  const int n = *e->host_n;
  if (n <= 0) return 0;
  if (n > L.n) return fail(AZ_E_DEVICE, "host evaluator: leaf count past the lane's slots");
  AZ_HIP(hipMemcpyAsync(e->host_x, L.x, (size_t)n * HW * 4 * sizeof(float), hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  if (e->host_fn(e->host_user, e->host_x, n, e->host_p, e->host_v) != 0)
    return fail(AZ_E_CALLBACK, "the host evaluator returned an error");
  AZ_HIP(hipMemcpyAsync(L.probs, e->host_p, (size_t)n * A * sizeof(float), hipMemcpyHostToDevice, s));
  AZ_HIP(hipMemcpyAsync(L.values, e->host_v, (size_t)n * sizeof(float), hipMemcpyHostToDevice, s));
  AZ_HIP(hipStreamSynchronize(s));  // the staging buffers are reused by the next lane
  return 0;
}

int sync_all(az_engine* e);

// one simulation for every active slot of a lane (MCTS.search body,
// mcts.py:171-180), enqueued on the lane's stream
int simulate(az_engine* e, Lane& L) {
  hipStream_t s = L.stream;
  L.t.epoch += 1;
  // leaf records of any other simulation read as absent: the tag is unique
  // over the engine's lanes; when it wraps (2^32 simulations) the records are
  // cleared first, so none written 2^32 simulations ago can match
  if (++e->leaf_epoch == 0) {
    if (int rc = sync_all(e)) return rc;
    AZ_HIP(hipMemset(e->t.leaf_src, 0, (size_t)e->g.slots * sizeof(uint64_t)));
    e->leaf_epoch = 1;
  }
  L.t.leaf_epoch = e->leaf_epoch;
  // eval_count, miss_count, nn_count: the epoch parity's block of
  // four (zeroed by the previous simulation's select kernel, or at creation)
  set_counts(L.t, L.counts, L.t.epoch & 1);
  if (L.tree_timer.enabled) L.tree_timer.begin(s);
  az::launch_select(L.g, L.t, e->cache, s);
  if (L.tree_timer.enabled) L.tree_timer.end(s, 1);
  const az::Board* rows = L.t.eval_board;
  const int32_t* n_rows = L.t.eval_count;
  if (e->cache.enabled) {  // the select launch resolved its duplicate boards (dedup_tail)
    rows = L.t.nn_board;
    n_rows = L.t.nn_count;
  }
  if (e->cfg.evaluator == AZ_EVAL_NETWORK) {
    // the stem reads the queued boards straight (no encode pass; bitwise the same outputs)
    az::launch_forward(e->net, L.x, n_rows, L.n, L.g.H, L.g.W, L.g.A, L.act[0], L.act[1], L.act[2],
                       L.probs, L.values, s, L.timer.enabled ? &L.timer : nullptr, rows);
  } else if (e->cfg.evaluator == AZ_EVAL_HOST) {
    if (int rc = host_evaluate(e, L, rows, n_rows)) {
      e->broken = true;
      return rc;
    }
  } else {
    az::launch_synth_eval(L.g, rows, n_rows, L.probs, L.values, s);
  }
  if (L.tree_timer.enabled) L.tree_timer.begin(s);
  az::launch_expand(L.g, L.t, e->cache, L.probs, L.values, s);
  if (L.tree_timer.enabled) L.tree_timer.end(s, 1);
  AZ_HIP(hipGetLastError());
  return 0;
}

int sync_all(az_engine* e) {
  AZ_HIP(hipStreamSynchronize(e->stream));
  for (hipStream_t s : e->lane_streams) AZ_HIP(hipStreamSynchronize(s));
  if (e->own_pack_stream) AZ_HIP(hipStreamSynchronize(e->pack_stream));
  return 0;
}

// Entry of an ABI call that reads or writes engine buffers: the device, then
// every queued move finished (az_selfplay_step without stats returns while
// the lanes' kernels run on non-blocking streams; their samples, trees and
// evaluator slices must not be read or overwritten under them).
int enter(az_engine* e) {
  AZ_HIP(hipSetDevice(e->device));
  return sync_all(e);
}

// the tree API never compacts (its views are the whole tree, like the
// reference's object graph): an engine created with compact = 1 sizes each
// arena half for one move, which a reused tree outgrows
int tree_api_ok(az_engine* e) {
  if (e->g.halves > 1)
    return fail(AZ_E_INVALID, "the tree API (az_tree_*) needs an engine created with compact = 0");
  return 0;
}

int cache_clear(az_engine* e) {
  if (!e->cache.state) return 0;
  int rc;
  if ((rc = sync_all(e))) return rc;
  AZ_HIP(hipMemsetAsync(e->cache.state, 0, ((size_t)e->cache.mask + 1) * sizeof(uint32_t), e->stream));
  AZ_HIP(hipMemsetAsync(e->cache.ctl, 0, 4 * sizeof(unsigned long long), e->stream));
  AZ_HIP(hipStreamSynchronize(e->stream));
  return 0;
}

int ready_to_search(az_engine* e) {
  if (e->broken)
    return fail(AZ_E_STATE, "a host evaluator error interrupted a simulation: the trees are incomplete "
                            "until az_selfplay_begin or az_tree_reset");
  if (e->cfg.evaluator == AZ_EVAL_NETWORK && !e->net.ready)
    return fail(AZ_E_STATE, "network evaluator selected but az_engine_set_weights was not called");
  if (e->cfg.evaluator == AZ_EVAL_HOST && !e->host_fn)
    return fail(AZ_E_STATE, "host evaluator selected but az_engine_set_evaluator was not called");
  return 0;
}

// ------------------------------------------------------------ weight folding
[[maybe_unused]] int fetch(const std::map<std::string, const az_tensor*>& m, const std::string& name,
          int64_t numel, std::vector<double>& out) {
  auto it = m.find(name);
  if (it == m.end()) return fail(AZ_E_INVALID, "missing weight tensor '" + name + "'");
  const az_tensor* t = it->second;
  if (t->numel != numel)
    return fail(AZ_E_INVALID, "weight '" + name + "' has " + std::to_string(t->numel) +
                                  " elements, expected " + std::to_string(numel));
  std::vector<float> tmp(numel);
  if (t->on_device) {
    AZ_HIP(hipMemcpy(tmp.data(), t->data, numel * sizeof(float), hipMemcpyDeviceToHost));
  } else {
    memcpy(tmp.data(), t->data, numel * sizeof(float));
  }
  out.assign(tmp.begin(), tmp.end());
  return 0;
}

// InnerConvBlock (base_layers.py:20-66): conv kernel [kh][kw][cin][cout] +
// bias, BatchNorm(gamma, beta, moving mean/var).  Returns the folded kernel in
// Keras layout (double) and folded bias.
[[maybe_unused]] int fold_unit(const std::map<std::string, const az_tensor*>& m, const std::string& u, int kk,
              int cin, int cout, double eps, std::vector<double>& w, std::vector<double>& b) {
  std::vector<double> gamma, beta, mean, var;
  int rc;
  if ((rc = fetch(m, u + ".kernel", (int64_t)kk * kk * cin * cout, w))) return rc;
  if ((rc = fetch(m, u + ".bias", cout, b))) return rc;
  if ((rc = fetch(m, u + ".gamma", cout, gamma))) return rc;
  if ((rc = fetch(m, u + ".beta", cout, beta))) return rc;
  if ((rc = fetch(m, u + ".mean", cout, mean))) return rc;
  if ((rc = fetch(m, u + ".var", cout, var))) return rc;
  for (int n = 0; n < cout; ++n) {
    const double sc = gamma[n] / sqrt(var[n] + eps);
    for (int i = 0; i < kk * kk * cin; ++i) w[(size_t)i * cout + n] *= sc;
    b[n] = (b[n] - mean[n]) * sc + beta[n];
  }
  return 0;
}

// [n][K] (K contiguous) -> MFMA fragment order of conv3x3_mfma_kernel:
// float4 index ((c*4 + tile)*4 + q)*64 + lane holds W[k][n] for
// k = 32c + 16*(lane>>5) + 4q + e (e = 0..3), n = 32*tile + (lane&31).
[[maybe_unused]] std::vector<float> pack_fragments(const std::vector<float>& wt, int N, int K) {
  std::vector<float> p((size_t)N * K);
  const int chunks = K / 32, tiles = N / 32;
  for (int c = 0; c < chunks; ++c)
    for (int t = 0; t < tiles; ++t)
      for (int q = 0; q < 4; ++q)
        for (int lane = 0; lane < 64; ++lane)
          for (int e = 0; e < 4; ++e) {
            const int k = 32 * c + 16 * (lane >> 5) + 4 * q + e;
            const int n = 32 * t + (lane & 31);
            p[((((size_t)c * tiles + t) * 4 + q) * 64 + lane) * 4 + e] = wt[(size_t)n * K + k];
          }
  return p;
}

// conv16_kernel pack (az_conv16.hip) of a folded 3x3 conv [3][3][cin][F] (+ the
// 1x1 residual [F][F]): fp16 bits, uploaded as raw storage; *scale = 2^(e-12)
[[maybe_unused]] int upload_conv16(std::vector<void*>& owned, uint16_t** dst, float* scale,
                                   const std::vector<double>& w3, int cin, const std::vector<double>* wr) {
  const int e = az::conv16_prescale(w3.data(), w3.size(), wr ? wr->data() : nullptr, wr ? wr->size() : 0);
  std::vector<uint16_t> pack;
  az::conv16_pack(w3.data(), cin, wr ? wr->data() : nullptr, e, pack);
  *scale = std::ldexp(1.f, e - 12);
  void* q = nullptr;
  AZ_HIP(hipMalloc(&q, pack.size() * sizeof(uint16_t)));
  owned.push_back(q);
  *dst = reinterpret_cast<uint16_t*>(q);
  AZ_HIP(hipMemcpy(q, pack.data(), pack.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  return 0;
}

[[maybe_unused]] int upload(std::vector<void*>& owned, float** dst, const std::vector<float>& src) {
  if (!*dst) {
    void* q = nullptr;
    AZ_HIP(hipMalloc(&q, std::max<size_t>(src.size(), 1) * sizeof(float)));
    owned.push_back(q);
    *dst = reinterpret_cast<float*>(q);
  }
  AZ_HIP(hipMemcpy(*dst, src.data(), src.size() * sizeof(float), hipMemcpyHostToDevice));
  return 0;
}

// Lane views: per-slot arrays offset to the lane's first slot; with more than
// one lane each gets its own eval-queue counters and dedup table.
int make_lane(az_engine* e, Lane* L, int first, int n, bool own_queue) {
  const az::GameCfg& g = e->g;
  L->first = first;
  L->n = n;
  L->g = g;
  L->g.slots = n;
  az::TreeDev t = e->t;
  const size_t f = (size_t)first;
  if (g.halves == 1) t.edges += f * g.arena_cap;  // pooled: the lane's own pool (alloc_pool)
  if (t.arena_end) t.arena_end += f;
  if (t.slot_live) t.slot_live += f;
  t.root_board += f;
  t.root_first += f;
  t.root_n += f;
  t.root_value += f;
  t.arena_top += f;
  t.ply += f;
  t.game_id += f;
  t.path += f * g.max_depth;
  t.path_len += f;
  t.slot_expansions += f;
  t.mt += f;  // word-major: stride stays the whole engine's slot count
  t.leaf_src += f;
  t.leaf_board += f;
  t.eval_board += f;

  t.nn_board += f;
  t.last_move += f;
  t.last_status += f;
  t.last_policy += f * g.A;
  if (own_queue) {
    int rc;
    if ((rc = e->alloc(&t.eval_count, az::kCountWords))) return rc;
    AZ_HIP(hipMemset(t.eval_count, 0, az::kCountWords * sizeof(int32_t)));
    set_counts(t, t.eval_count, 0);
    t.epoch = 0;
  }
  L->counts = t.eval_count;
  L->t = t;
  L->x = e->x + f * g.HW * 4;
  for (int i = 0; i < 3; ++i) L->act[i] = e->act[i] ? e->act[i] + f * g.HW * 128 : nullptr;
  L->probs = e->probs + f * g.A;
  L->values = e->values + f;
  return 0;
}

// compacted self-play: the lane's two pool halves of `cap` edges and their counters
int alloc_pool(az_engine* e, Lane* L, int64_t cap) {
  int rc;
  az::Edge* halves = nullptr;
  unsigned long long* tops = nullptr;
  if ((rc = e->alloc(&halves, 2 * (size_t)cap)) || (rc = e->alloc(&tops, 2))) return rc;
  AZ_HIP(hipMemset(tops, 0, 2 * sizeof(unsigned long long)));
  L->pool_cap = cap;
  L->t.pool_cap = (int32_t)cap;
  L->t.edges = halves;
  L->t.dst_edges = halves + cap;
  L->t.pool_top = tops;
  L->t.dst_top = tops + 1;
  return 0;
}

}  // namespace

namespace az {
// Folds (BatchNorm into conv) and uploads the network weights, Keras names
// of custom_alphazero/model/weights.py.  in_ch = 4: the Connect-N stem
// kernels (stem_w [36][F]; the one-launch tower's stem16 pack and its
// small-weight blob); in_ch > 4 (chess, 118 planes): the stem is one more
// conv16 3x3 conv over the input zero-padded to F channels (stem_k).
int load_network(NetDev& net, const az_tensor* tensors, int n, int in_ch, int HW, int A, double eps,
                 std::vector<void*>& owned) {
  std::map<std::string, const az_tensor*> m;
  for (int i = 0; i < n; ++i) {
    if (!tensors[i].name || !tensors[i].data) return fail(AZ_E_INVALID, "tensor without name/data");
    m[tensors[i].name] = &tensors[i];
  }
  const int F = 128, hidden = net.hidden;
  if (in_ch < 1 || in_ch > F) return fail(AZ_E_INVALID, "input planes must be 1..128");
  std::vector<double> w, b, wr, br;
  int rc;
  if ((rc = fold_unit(m, "stem", 3, in_ch, F, eps, w, b))) return rc;
  // host copies for the one-launch tower (tower16_kernel): its stem pack and the small-weight blob
  // (in_ch > 4, chess: the input-row form, whose stem is the conv16 pack stem_k)
  const bool tower = net.use_tower && (in_ch == 4 || HW == 64);
  const bool rows_tower = tower && in_ch > 4;
  std::vector<float> tb_b1, tb_b2, tb_stemb(b.begin(), b.end()), tb_pcw, tb_vcw, tb_hb(4, 0.f), tb_pdw, tb_pdb,
      tb_v1w, tb_v1b, tb_v2w;
  uint16_t* stem16 = nullptr;
  float stem_s = 1.f;
  if (tower && !rows_tower) {
    const int e = conv16_prescale(w.data(), w.size(), nullptr, 0);
    std::vector<uint16_t> pack;
    tower16_stem_pack(w.data(), e, pack);
    stem_s = std::ldexp(1.f, e - 12);
    void* q = nullptr;
    AZ_HIP(hipMalloc(&q, pack.size() * sizeof(uint16_t)));
    owned.push_back(q);
    stem16 = reinterpret_cast<uint16_t*>(q);
    AZ_HIP(hipMemcpy(q, pack.data(), pack.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  }
  {
    std::vector<float> bs(F);
    for (int i = 0; i < F; ++i) bs[i] = (float)b[i];
    if ((rc = upload(owned, &net.stem_b, bs))) return rc;
    if (in_ch == 4) {  // [3][3][4][F] -> [tap*4 + c][F]
      std::vector<float> ws(36 * F);
      for (int i = 0; i < 36 * F; ++i) ws[i] = (float)w[i];  // Keras order == (tap, c, n)
      if ((rc = upload(owned, &net.stem_w, ws))) return rc;
    } else {  // [3][3][in_ch][F]: the conv16 pack pads the channels; direct: [3][3][F][F] zero-padded
      if ((rc = upload_conv16(owned, &net.stem_k, &net.stem_scale, w, in_ch, nullptr))) return rc;
      std::vector<float> wt((size_t)F * 9 * F, 0.f);
      for (int tap = 0; tap < 9; ++tap)
        for (int c = 0; c < in_ch; ++c)
          for (int o = 0; o < F; ++o) wt[(size_t)o * 9 * F + tap * F + c] = (float)w[((size_t)tap * in_ch + c) * F + o];
      if ((rc = upload(owned, &net.stem_d, pack_fragments(wt, F, 9 * F)))) return rc;
    }
    net.in_ch = in_ch;
  }
  net.c1_w.assign(net.depth, nullptr);
  net.c1_b.assign(net.depth, nullptr);
  net.c2_w.assign(net.depth, nullptr);
  net.c2_b.assign(net.depth, nullptr);
  net.k1.assign(net.depth, nullptr);
  net.k2.assign(net.depth, nullptr);
  net.k1_scale.assign(net.depth, 1.f);
  net.k2_scale.assign(net.depth, 1.f);
  for (int d = 0; d < net.depth; ++d) {
    const std::string p = "block" + std::to_string(d);
    if ((rc = fold_unit(m, p + ".conv1", 3, F, F, eps, w, b))) return rc;
    std::vector<float> wt((size_t)F * 9 * F), bt(F);
    for (int n2 = 0; n2 < F; ++n2)
      for (int k = 0; k < 9 * F; ++k) wt[(size_t)n2 * 9 * F + k] = (float)w[(size_t)k * F + n2];
    for (int i = 0; i < F; ++i) bt[i] = (float)b[i];
    tb_b1.insert(tb_b1.end(), bt.begin(), bt.end());
    if ((rc = upload(owned, &net.c1_w[d], pack_fragments(wt, F, 9 * F))) ||
        (rc = upload_conv16(owned, &net.k1[d], &net.k1_scale[d], w, F, nullptr)) ||
        (rc = upload(owned, &net.c1_b[d], bt)))
      return rc;
    if ((rc = fold_unit(m, p + ".conv2", 3, F, F, eps, w, b))) return rc;
    if ((rc = fold_unit(m, p + ".res", 1, F, F, eps, wr, br))) return rc;
    std::vector<float> wt2((size_t)F * 10 * F), bt2(F);
    for (int n2 = 0; n2 < F; ++n2) {
      for (int k = 0; k < 9 * F; ++k) wt2[(size_t)n2 * 10 * F + k] = (float)w[(size_t)k * F + n2];
      for (int c = 0; c < F; ++c) wt2[(size_t)n2 * 10 * F + 9 * F + c] = (float)wr[(size_t)c * F + n2];
    }
    for (int i = 0; i < F; ++i) bt2[i] = (float)(b[i] + br[i]);
    tb_b2.insert(tb_b2.end(), bt2.begin(), bt2.end());
    if ((rc = upload(owned, &net.c2_w[d], pack_fragments(wt2, F, 10 * F))) ||
        (rc = upload_conv16(owned, &net.k2[d], &net.k2_scale[d], w, F, &wr)) ||
        (rc = upload(owned, &net.c2_b[d], bt2)))
      return rc;
  }
  // heads
  if ((rc = fold_unit(m, "policy.conv", 1, F, 2, eps, w, b))) return rc;
  {
    std::vector<float> a(w.begin(), w.end()), c(b.begin(), b.end());
    tb_pcw = a;
    tb_hb[0] = c[0];
    tb_hb[1] = c[1];
    if ((rc = upload(owned, &net.pc_w, a)) || (rc = upload(owned, &net.pc_b, c))) return rc;
  }
  if ((rc = fold_unit(m, "value.conv", 1, F, 1, eps, w, b))) return rc;
  {
    std::vector<float> a(w.begin(), w.end()), c(b.begin(), b.end());
    tb_vcw = a;
    tb_hb[2] = c[0];
    if ((rc = upload(owned, &net.vc_w, a)) || (rc = upload(owned, &net.vc_b, c))) return rc;
  }
  struct DenseSpec {
    const char* name;
    int in, out;
    float** w;
    float** b;
  } dense[] = {{"policy.dense", 2 * HW, A, &net.pd_w, &net.pd_b},
               {"value.dense1", HW, hidden, &net.v1_w, &net.v1_b},
               {"value.dense2", hidden, 1, &net.v2_w, &net.v2_b}};
  for (auto& ds : dense) {
    if ((rc = fetch(m, std::string(ds.name) + ".kernel", (int64_t)ds.in * ds.out, w))) return rc;
    if ((rc = fetch(m, std::string(ds.name) + ".bias", ds.out, b))) return rc;
    std::vector<float> a(w.begin(), w.end()), c(b.begin(), b.end());
    if ((rc = upload(owned, ds.w, a)) || (rc = upload(owned, ds.b, c))) return rc;
    if (ds.w == &net.pd_w) {
      tb_pdw = a;
      tb_pdb = c;
    } else if (ds.w == &net.v1_w) {
      tb_v1w = a;
      tb_v1b = c;
    } else {
      tb_v2w = a;
      tb_hb[3] = c[0];
    }
    if (ds.w == &net.pd_w && A > kMaxActions) {
      const int K = ds.in, tiles = (A + 63) / 64;
      std::vector<float> t((size_t)tiles * K * 64, 0.f);
      for (int k = 0; k < K; ++k)
        for (int o = 0; o < A; ++o) t[((size_t)(o / 64) * K + k) * 64 + (o % 64)] = a[(size_t)k * A + o];
      if ((rc = upload(owned, &net.pd_wt, t))) return rc;
    }
  }
  if (tower) {
    TowerNet tn{};
    for (int d = 0; d < net.depth; ++d) {
      tn.k1[d] = reinterpret_cast<const uint4*>(net.k1[d]);
      tn.k2[d] = reinterpret_cast<const uint4*>(net.k2[d]);
      tn.s1[d] = net.k1_scale[d];
      tn.s2[d] = net.k2_scale[d];
    }
    tn.stem16 = reinterpret_cast<const uint4*>(stem16);
    tn.stem_s = stem_s;
    tn.stem_k = rows_tower ? reinterpret_cast<const uint4*>(net.stem_k) : nullptr;
    tn.stem_ks = net.stem_scale;
    // the small-weight blob (TowerNet), every part padded to a multiple of 4 floats
    std::vector<float> blob;
    auto put = [&](const std::vector<float>& v) {
      const int off = (int)blob.size();
      blob.insert(blob.end(), v.begin(), v.end());
      while (blob.size() % 4) blob.push_back(0.f);
      return off;
    };
    tn.off_b1 = put(tb_b1);
    tn.off_b2 = put(tb_b2);
    tn.off_stemb = put(tb_stemb);
    tn.off_wpc = put(tb_pcw);
    tn.off_wvc = put(tb_vcw);
    tn.off_hb = put(tb_hb);
    tn.off_bpd = put(tb_pdb);
    tn.off_bv1 = put(tb_v1b);
    tn.off_wv2 = put(tb_v2w);
    tn.off_wpd = put(tb_pdw);
    tn.off_wv1 = put(tb_v1w);
    tn.blob_floats = (int)blob.size();
    // the layout: 128/96-row tiles double-buffered, else one tile in place;
    // per layout the largest staging that fits: the whole blob, then without
    // wv1, then without wpd too (those then read from L2)
    // (the input-row form runs no dense head: the biases and 1x1 head weights only)
    const int prefix[3] = {rows_tower ? tn.off_bpd : tn.blob_floats, tn.off_wv1, tn.off_wpd};
    struct Layout {
      int tr;
      bool db;
    } layouts[2] = {{tower16_tile_rows(HW), true}, {tower16_tile_rows(HW), false}};
    bool found = false;
    for (int li = 0; li < 2 && !found; ++li) {
      const Layout L = layouts[li];
      if (!L.tr || (!rows_tower && !tower16_heads_fit(HW, L.tr, A, net.hidden, L.db))) continue;
      if (rows_tower && (L.tr != 128 || tower16_lds_bytes(HW, L.tr, prefix[0], L.db) > kTowerLdsMax)) continue;
      for (int i = 0; i < (rows_tower ? 1 : 3) && !found; ++i)
        if (tower16_lds_bytes(HW, L.tr, prefix[i], L.db) <= kTowerLdsMax) {
          tn.tile_rows = L.tr;
          tn.dbuf = L.db;
          tn.staged_floats = prefix[i];
          tn.wv1_lds = i == 0 && !rows_tower;
          tn.wpd_lds = i <= 1 && !rows_tower;
          found = true;
        }
    }
    if (!found) {  // the per-layer kernels instead (same arithmetic)
      net.use_tower = false;
      if (net.board_w > 16) net.algo = AZ_CONV_DIRECT;
      net.ready = true;
      return 0;
    }
    tn.wv1_xtile = !rows_tower && tn.dbuf && !tn.wv1_lds && tower16_wv1_xtile_fits(HW, tn.tile_rows, net.hidden);
    // the slot plan: border blocks skip the taps past their edge
    // (az_config.tower_natural_order: natural order, no skips -- bitwise the same outputs)
    {
      std::vector<int> pix;
      int skip[2] = {0, 0};
      if (!net.tower_natural_order && net.board_h * net.board_w == HW)
        tower16_slot_plan(net.board_h, net.board_w, tn.tile_rows, pix, skip);
      tn.slot_pix = nullptr;
      tn.skip[0] = skip[0];
      tn.skip[1] = skip[1];
      if (!pix.empty()) {
        void* q = nullptr;
        AZ_HIP(hipMalloc(&q, pix.size() * sizeof(int)));
        owned.push_back(q);
        AZ_HIP(hipMemcpy(q, pix.data(), pix.size() * sizeof(int), hipMemcpyHostToDevice));
        tn.slot_pix = reinterpret_cast<const int*>(q);
      }
    }
    // dual launches (tower16_dual_kernel): boards of 33-48 cells (Connect-4)
    // in 128-row tiles of three may also run 96-row tiles of two, with a
    // slot plan of their own, when a launch holds at most two boards per CU
    // that the lanes' towers leave each other (2 * CUs / lanes: Connect-4 at
    // configs[1], ~120 live boards per lane launch with the LRU cache, gains
    // 4.4%; at 373 or 1113 boards the 96-row tiles lose 20%, profiles/r6/)
    tn.alt_rows = 0;
    tn.alt_slot_pix = nullptr;
    tn.alt_skip[0] = tn.alt_skip[1] = 0;
    tn.alt_max_boards = -1;
    tn.alt_staged_floats = tn.alt_wpd_lds = tn.alt_wv1_lds = 0;
    if (!rows_tower && tn.tile_rows == 128 && tn.dbuf && tower16_boards_per_tile(HW, 128) == 3 &&
        tower16_boards_per_tile(HW, 96) == 2 && tower16_heads_fit(HW, 96, A, net.hidden, true)) {
      int dev = 0, cus = 0;
      AZ_HIP(hipGetDevice(&dev));
      AZ_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      tn.alt_rows = 96;
      tn.alt_max_boards = 2 * std::max(1, cus / std::max(1, net.lanes));
      // the largest staging the 96-row layout holds (it has 64 rows fewer
      // than the 128-row one: the whole blob, where 128 rows leave wv1 in L2)
      for (int i = 0; i < 3; ++i)
        if (tower16_lds_bytes(HW, 96, prefix[i], true) <= kTowerLdsMax) {
          tn.alt_staged_floats = prefix[i];
          tn.alt_wv1_lds = i == 0;
          tn.alt_wpd_lds = i <= 1;
          break;
        }
      std::vector<int> pix;
      int skip[2] = {0, 0};
      if (!net.tower_natural_order && net.board_h * net.board_w == HW)
        tower16_slot_plan(net.board_h, net.board_w, 96, pix, skip);
      tn.alt_skip[0] = skip[0];
      tn.alt_skip[1] = skip[1];
      if (!pix.empty()) {
        void* q = nullptr;
        AZ_HIP(hipMalloc(&q, pix.size() * sizeof(int)));
        owned.push_back(q);
        AZ_HIP(hipMemcpy(q, pix.data(), pix.size() * sizeof(int), hipMemcpyHostToDevice));
        tn.alt_slot_pix = reinterpret_cast<const int*>(q);
      }
    }
    tn.depth = net.depth;
    tn.hidden = net.hidden;
    if (!net.tower) {
      void* q = nullptr;
      AZ_HIP(hipMalloc(&q, sizeof(TowerNet)));
      owned.push_back(q);
      net.tower = reinterpret_cast<TowerNet*>(q);
    }
    void* qb = nullptr;
    AZ_HIP(hipMalloc(&qb, blob.size() * sizeof(float)));
    owned.push_back(qb);
    AZ_HIP(hipMemcpy(qb, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice));
    tn.blob = reinterpret_cast<const float*>(qb);
    AZ_HIP(hipMemcpy(net.tower, &tn, sizeof(TowerNet), hipMemcpyHostToDevice));
    net.tower_staged = tn.staged_floats;
    net.tower_dbuf = tn.dbuf != 0;
    net.tower_rows = tn.tile_rows;
    net.tower_alt_rows = tn.alt_rows;
    net.tower_alt_staged = tn.alt_staged_floats;
    // (chess: as self-play runs it, the stem's known-zero input chunks 0-1 skipped)
    net.issued_flop_per_board = tower16_issued_flop_per_board(HW, tn.tile_rows, net.depth, tn.skip, rows_tower, 2);
    net.issued_flop_per_board_small =
        tn.alt_rows ? tower16_issued_flop_per_board(HW, tn.alt_rows, net.depth, tn.alt_skip, rows_tower, 2) : 0.0;
    net.tower_small_max_boards = tn.alt_rows ? tn.alt_max_boards : -1;
  }
  net.ready = true;
  return 0;
}
}  // namespace az

extern "C" {

int az_abi_version(void) { return AZ_ABI_VERSION; }
#ifndef AZ_SRC_HASH
#define AZ_SRC_HASH "unknown"
#endif
#ifndef AZ_BUILD_EXTRA
#define AZ_BUILD_EXTRA "unknown"
#endif
const char* az_build_id(void) { return AZ_SRC_HASH; }
const char* az_build_flags(void) { return AZ_BUILD_EXTRA; }
const char* az_last_error(void) { return g_last_error.c_str(); }

int az_engine_create(int device, const az_config* cfg, az_engine** out) {
  if (!cfg || !out) return fail(AZ_E_INVALID, "null argument");
  const az_config& c = *cfg;
  if (c.board_height < 2 || c.board_width < 2 || c.board_height * c.board_width > az::kMaxCells)
    return fail(AZ_E_INVALID, "board must have 4..128 cells");
  if (c.n < 2 || c.n > std::min(c.board_height, c.board_width))
    return fail(AZ_E_INVALID, "need 2 <= n <= min(width, height) (connect_n/board.py:14-18)");
  const int A = c.gravity ? c.board_width : c.board_width * c.board_height;
  if (A > az::kMaxActions) return fail(AZ_E_INVALID, "action space too large");
  if (c.slots < 1 || c.mcts_iterations < 1) return fail(AZ_E_INVALID, "slots and mcts_iterations must be >= 1");
  if (c.conv_algo != AZ_CONV_F16X2 && c.conv_algo != AZ_CONV_DIRECT && c.conv_algo != AZ_CONV_F16X2_LAYERS)
    return fail(AZ_E_INVALID, "conv_algo must be AZ_CONV_F16X2, AZ_CONV_DIRECT or AZ_CONV_F16X2_LAYERS");
  if (c.evaluator == AZ_EVAL_NETWORK && c.conv_algo == AZ_CONV_F16X2_LAYERS && c.board_width > 16)
    return fail(AZ_E_INVALID, "AZ_CONV_F16X2_LAYERS supports boards up to 16 columns");
  if (c.depth < 0 || c.depth > 1024 || c.value_hidden < 1) return fail(AZ_E_INVALID, "need 0 <= depth and value_hidden >= 1");
  if (c.evaluator == AZ_EVAL_NETWORK && (int64_t)c.slots * c.board_height * c.board_width * 512 >= (1ll << 31))
    return fail(AZ_E_INVALID, "slots * H * W * 512 must stay below 2^31 (32-bit activation byte offsets)");
  if (c.evaluator != AZ_EVAL_NETWORK && c.evaluator != AZ_EVAL_SYNTHETIC && c.evaluator != AZ_EVAL_HOST)
    return fail(AZ_E_INVALID, "unknown evaluator");
  if (c.evaluator == AZ_EVAL_NETWORK && c.filters != 128)
    return fail(AZ_E_INVALID, "network evaluator supports filters == 128 (ConfigModel.filters)");
  int dev_count = 0;
  if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count == 0)
    return fail(AZ_E_HIP, "no HIP device visible: libaz has no CPU fallback");
  if (device < 0 || device >= dev_count) return fail(AZ_E_INVALID, "bad device index");
  AZ_HIP(hipSetDevice(device));

  az_engine* e = new az_engine();
  e->device = device;
  e->cfg = c;
  az::GameCfg& g = e->g;
  g.H = c.board_height;
  g.W = c.board_width;
  g.HW = g.H * g.W;
  g.n = c.n;
  g.gravity = c.gravity ? 1 : 0;
  g.A = A;
  g.sims = c.mcts_iterations;
  g.greedy_ply = c.index_move_greedy;
  g.c_puct = c.exploration_constant;
  g.slots = c.slots;
  g.max_depth = g.HW + 1;
  g.noise = c.dirichlet_noise != 0;
  g.noise_alpha = c.dirichlet_alpha;
  g.noise_ratio = c.dirichlet_ratio;
  g.rng_skip = c.rng_skip;
  if (c.rng_skip < 0) {
    delete e;
    return fail(AZ_E_INVALID, "rng_skip must be >= 0");
  }
  if (g.noise && !(c.dirichlet_alpha > 0.0 && c.dirichlet_alpha <= 1.0 && std::isfinite(c.dirichlet_ratio))) {
    delete e;
    return fail(AZ_E_INVALID, "Dirichlet noise needs 0 < dirichlet_alpha <= 1 (the reference's 0.03) and a "
                              "finite dirichlet_ratio");
  }
  const int64_t visits = c.max_tree_visits > 0 ? c.max_tree_visits : (int64_t)c.mcts_iterations * g.HW + 2;
  // a slot's tree holds at most mcts_iterations * H*W expansions of <= A edges
  // (one game): `safe` edges per slot can never overflow.
  //  * uncompacted (tree API): a static run of arena_edges (default safe) per slot;
  //  * compacted self-play (az_config.compact): pooled arenas (az_tree.h) -- per
  //    lane two halves of arena_edges x the lane's slots, arena_edges (an
  //    average per slot) defaulting to safe when two such halves per slot fit
  //    in 40% of the free HBM, else the most that does (at least 8 S A + H W A).
  //    A slot holds what it uses -- one move's search plus its kept subtree,
  //    a few thousand edges at configs[1] -- so the pool is shared: a game
  //    whose kept subtree grows toward the whole game's search (a peaked
  //    network) takes the room other slots leave.  Overflow is kErrArena,
  //    never an overrun.
  g.halves = c.compact ? 2 : 1;
  const int64_t safe = (int64_t)c.mcts_iterations * g.HW * A + A;
  int64_t arena = c.arena_edges > 0 ? c.arena_edges : safe;
  if (c.arena_edges <= 0 && c.compact) {
    size_t free_b = 0, total_b = 0;
    if (hipSetDevice(device) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
      const int64_t fit = (int64_t)(0.4 * (double)free_b / ((double)c.slots * 2.0 * sizeof(az::Edge)));
      arena = std::min(safe, std::max(fit, (int64_t)8 * c.mcts_iterations * A + (int64_t)g.HW * A));
    }
  }
  if (visits > (1 << 30) || arena > (1 << 30) || (c.compact && arena < 2 * az::kPoolChunkA * A)) {
    delete e;
    return fail(AZ_E_INVALID, "tree bounds too large (or a pooled arena below two chunks per slot)");
  }
  g.pow_len = (int)visits;
  g.arena_cap = (int)arena;

  auto cleanup = [&](int rc) {
    az_engine_destroy(e);
    return rc;
  };
  int rc;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(AZ_E_HIP, "hipStreamCreate failed"));
  if (c.lanes < 0) return cleanup(fail(AZ_E_INVALID, "lanes must be >= 0"));
  const size_t S = (size_t)g.slots;
  az::TreeDev& t = e->t;
  t.edges = nullptr;
  t.arena_end = t.slot_live = nullptr;
  if (g.halves == 1 && (rc = e->alloc(&t.edges, S * (size_t)g.arena_cap))) return cleanup(rc);
  if (g.halves > 1 && ((rc = e->alloc(&t.arena_end, S)) || (rc = e->alloc(&t.slot_live, S)))) return cleanup(rc);
  if ((rc = e->alloc(&t.root_board, S)) ||
      (rc = e->alloc(&t.root_first, S)) || (rc = e->alloc(&t.root_n, S)) ||
      (rc = e->alloc(&t.root_value, S)) || (rc = e->alloc(&t.arena_top, S)) ||
      (rc = e->alloc(&t.ply, S)) || (rc = e->alloc(&t.game_id, S)) ||
      (rc = e->alloc(&t.path, S * g.max_depth)) || (rc = e->alloc(&t.path_len, S)) ||
      (rc = e->alloc(&t.slot_expansions, S)) || (rc = e->alloc(&t.mt, S * (az::kMtN + 1))) ||
      (rc = e->alloc(&t.leaf_src, S)) || (rc = e->alloc(&t.leaf_board, S)) ||
      (rc = e->alloc(&t.eval_board, S)) || (rc = e->alloc(&t.nn_board, S)) ||
      (rc = e->alloc(&t.eval_count, az::kCountWords)) || (rc = e->alloc(&t.stats, az::kStatCount)) ||
      (rc = e->alloc(&t.last_move, S)) || (rc = e->alloc(&t.last_status, S)) ||
      (rc = e->alloc(&t.last_policy, S * A)))
    return cleanup(rc);
  double* powtab = nullptr;
  if ((rc = e->alloc(&powtab, g.pow_len))) return cleanup(rc);
  {
    std::vector<double> h(g.pow_len);
    for (int k = 0; k < g.pow_len; ++k) h[k] = k == 0 ? 0.0 : g_pow((double)k, 0.5);
    if (hipMemcpy(powtab, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(fail(AZ_E_HIP, "pow table upload failed"));
  }
  t.powtab = powtab;
  t.mt_stride = g.slots;
  set_counts(t, t.eval_count, 0);
  t.epoch = 0;
  // leaf records start untagged (leaf_epoch counts from 1)
  if (hipMemset(t.leaf_src, 0, S * sizeof(uint64_t)) != hipSuccess)
    return cleanup(fail(AZ_E_HIP, "memset failed"));
  if (c.cache_log2 < 0 || c.cache_log2 > 30 || (c.cache_log2 > 0 && c.cache_log2 < 4))
    return cleanup(fail(AZ_E_INVALID, "cache_log2 must be 0 (no cache) or 4..30"));
  if (c.cache_log2 > 0) {
    const size_t cap = (size_t)1 << c.cache_log2;
    az::CacheDev& cd = e->cache;
    if ((rc = e->alloc(&cd.keys, cap)) || (rc = e->alloc(&cd.state, cap)) ||
        (rc = e->alloc(&cd.pay, cap * (A + 1))) || (rc = e->alloc(&cd.ctl, 4)))
      return cleanup(rc);
    cd.mask = (uint32_t)(cap - 1);
    cd.enabled = 1;
    // LRU eviction by generations of cap/kCacheGenDiv inserts -- or, for a
    // larger batch, of more than three moves of every slot's inserts (the
    // lane-drift bound, az_tree.h: configs[2]'s 8192 x S=200 and configs[3]'s
    // 4096 x S=400 need it at 2^26 entries) while at most cap/4 (four
    // generations per turnover keep the LRU order meaningful); otherwise the
    // table only fills (entries are never overwritten)
    const unsigned long long bound = 3ull * (unsigned long long)g.slots * (unsigned long long)g.sims + 1;
    const unsigned long long gen = std::max<unsigned long long>(cap / az::kCacheGenDiv, bound);
    cd.gen_size = gen <= cap / 4 ? gen : 0;
    if (hipMemset(cd.state, 0, cap * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(cd.ctl, 0, 4 * sizeof(unsigned long long)) != hipSuccess)
      return cleanup(fail(AZ_E_HIP, "cache memset failed"));
  }
  if (hipMemset(t.stats, 0, az::kStatCount * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(t.eval_count, 0, az::kCountWords * sizeof(int32_t)) != hipSuccess ||

      hipMemset(t.game_id, 0xff, S * sizeof(int64_t)) != hipSuccess)
    return cleanup(fail(AZ_E_HIP, "memset failed"));
  // evaluator buffers (batch = slots)
  if ((rc = e->alloc(&e->probs, S * A)) || (rc = e->alloc(&e->values, S)) ||
      (rc = e->alloc(&e->uniforms, S)) || (rc = e->alloc(&e->dev_i32, S)) ||
      (rc = e->alloc(&e->dev_boards, S)))
    return cleanup(rc);
  if ((rc = e->alloc(&e->x, S * g.HW * 4))) return cleanup(rc);
  if (c.evaluator == AZ_EVAL_HOST) {
    if (hipHostMalloc(&e->host_x, (size_t)S * g.HW * 4 * sizeof(float), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&e->host_p, (size_t)S * A * sizeof(float), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&e->host_v, (size_t)S * sizeof(float), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&e->host_n, sizeof(int32_t), hipHostMallocDefault) != hipSuccess)
      return cleanup(fail(AZ_E_HIP, "host evaluator staging allocation failed"));
  }
  if (c.evaluator == AZ_EVAL_NETWORK) {
    const size_t act = S * g.HW * 128;
    for (int i = 0; i < 3; ++i)
      if ((rc = e->alloc(&e->act[i], act))) return cleanup(rc);
  }
  e->net.depth = c.depth;
  e->net.board_h = g.H;
  e->net.board_w = g.W;
  e->net.algo = c.conv_algo == AZ_CONV_F16X2_LAYERS ? AZ_CONV_F16X2 : c.conv_algo;
  // AZ_CONV_F16X2: the one-launch tower when the network fits it (1 <= depth
  // <= 16, value_hidden <= 256, the head weights in LDS: load_network),
  // otherwise quietly the same arithmetic per layer -- or, where the per-layer
  // kernels do not apply (depth 0: the heads are fused into the last conv2;
  // boards wider than 16), the fp32 MFMA path; every form within NET_TOL
  e->net.use_tower = c.conv_algo == AZ_CONV_F16X2 && c.depth >= 1 && c.depth <= az::kTowerMaxDepth &&
                     c.value_hidden <= 256;
  e->net.tower_natural_order = c.tower_natural_order != 0;
  if (c.depth == 0 || (c.conv_algo != AZ_CONV_DIRECT && !e->net.use_tower && c.board_width > 16))
    e->net.algo = AZ_CONV_DIRECT;
  e->net.err = e->t.stats + az::kStatErrors;
  // lanes: 0 = auto (two streams once each lane still holds a few hundred
  // games; three for 1536-4096 slots when HIP gives the process a hardware
  // queue per stream -- with 4 a third lane shares one and loses 27%:
  // profiles/r5/ab_queues_lanes.txt; larger launches keep two)
  int nl = c.lanes;
  if (nl <= 0) {
    const int queues = g_hw_queues_at_load;
    nl = g.slots < 512 ? 1 : (queues >= 8 && g.slots >= 1536 && g.slots <= 4096) ? 3 : 2;
  }
  nl = std::min(nl, std::min(g.slots, 8));
  if ((rc = make_lane(e, &e->whole, 0, g.slots, false))) return cleanup(rc);
  e->whole.stream = e->stream;
  if (nl == 1) {
    e->lanes.push_back(&e->whole);
  } else {
    for (int l = 0; l < nl; ++l) {
      Lane* L = new Lane();
      e->lanes.push_back(L);
      const int lo = (int)((int64_t)g.slots * l / nl), hi = (int)((int64_t)g.slots * (l + 1) / nl);
      if ((rc = make_lane(e, L, lo, hi - lo, true))) return cleanup(rc);
      hipStream_t st;
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
        return cleanup(fail(AZ_E_HIP, "hipStreamCreate failed"));
      e->lane_streams.push_back(st);
      L->stream = st;
      for (hipEvent_t& ev : L->move_done)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
          return cleanup(fail(AZ_E_HIP, "hipEventCreate failed"));
    }
  }
  e->net.lanes = (int)e->lanes.size();  // (the tower's dual-launch threshold, load_network)
  if (g.halves > 1)  // pooled arenas, one pool per lane (whose indices stay below 2^31)
    for (Lane* L : e->lanes)
      if ((rc = alloc_pool(e, L, std::min<int64_t>((int64_t)g.arena_cap * L->n, (1ll << 31) - 1))))
        return cleanup(rc);
  if (nl == 1)
    for (hipEvent_t& ev : e->whole.move_done)
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
        return cleanup(fail(AZ_E_HIP, "hipEventCreate failed"));
  // drain: one lane runs on `stream`, so the pack needs a stream of its own;
  // with more lanes `stream` is idle while moves run
  e->own_pack_stream = nl == 1;
  if (e->own_pack_stream) {
    if (hipStreamCreateWithFlags(&e->pack_stream, hipStreamNonBlocking) != hipSuccess)
      return cleanup(fail(AZ_E_HIP, "hipStreamCreate failed"));
  } else {
    e->pack_stream = e->stream;
  }
  if ((rc = e->alloc(&e->move_arrive, 4))) return cleanup(rc);
  if (hipMemset(e->move_arrive, 0, 4 * sizeof(int32_t)) != hipSuccess ||
      hipHostMalloc(&e->snap_host, 4 * sizeof(unsigned long long), hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&e->snap_dev, e->snap_host, 0) != hipSuccess)
    return cleanup(fail(AZ_E_HIP, "drain snapshot setup failed"));
  for (int i = 0; i < 4; ++i) e->snap_host[i] = 0;
  e->net.hidden = c.value_hidden;
  *out = e;
  return 0;
}

int az_engine_lanes(const az_engine* eng) { return eng ? (int)eng->lanes.size() : 0; }

int az_engine_destroy(az_engine* eng) {
  if (!eng) return 0;
  (void)hipSetDevice(eng->device);
  if (eng->stream) (void)hipStreamSynchronize(eng->stream);
  for (hipStream_t s : eng->lane_streams) {
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
  }
  if (eng->own_pack_stream && eng->pack_stream) {
    (void)hipStreamSynchronize(eng->pack_stream);
    (void)hipStreamDestroy(eng->pack_stream);
  }
  if (eng->snap_host) (void)hipHostFree(eng->snap_host);
  for (Lane* L : eng->lanes) {
    for (hipEvent_t ev : L->move_done)
      if (ev) (void)hipEventDestroy(ev);
    if (L != &eng->whole) delete L;
  }
  if (eng->lanes.size() > 1)
    for (hipEvent_t ev : eng->whole.move_done)
      if (ev) (void)hipEventDestroy(ev);
  if (eng->drain_dev) (void)hipFree(eng->drain_dev);
  if (eng->drain_host) (void)hipHostFree(eng->drain_host);
  for (void* p : eng->sample_bufs) (void)hipFree(p);
  for (void* p : eng->owned) (void)hipFree(p);
  if (eng->timer_ref) (void)hipEventDestroy(eng->timer_ref);
  for (void* q : {(void*)eng->host_x, (void*)eng->host_p, (void*)eng->host_v, (void*)eng->host_n})
    if (q) (void)hipHostFree(q);
  if (eng->stream) (void)hipStreamDestroy(eng->stream);
  delete eng;
  return 0;
}

int az_engine_set_evaluator(az_engine* e, az_eval_fn fn, void* user) {
  if (!e || !fn) return fail(AZ_E_INVALID, "null argument");
  if (e->cfg.evaluator != AZ_EVAL_HOST) return fail(AZ_E_STATE, "the engine was not created with AZ_EVAL_HOST");
  if (int rc_ = enter(e)) return rc_;
  e->host_fn = fn;
  e->host_user = user;
  return cache_clear(e);  // cached outputs belong to the previous evaluator
}

int az_engine_set_weights(az_engine* e, const az_tensor* tensors, int n) {
  if (!e || (!tensors && n)) return fail(AZ_E_INVALID, "null argument");
  if (int rc_ = enter(e)) return rc_;
  int rc;
  if ((rc = az::load_network(e->net, tensors, n, 4, e->g.HW, e->g.A, e->cfg.bn_epsilon, e->owned)))
    return rc;
  return cache_clear(e);  // cached outputs belong to the previous weights
}

int az_encode(az_engine* e, const int8_t* boards, int n, float* state, uint8_t* mask) {
  if (!e || n < 0 || (n && !boards)) return fail(AZ_E_INVALID, "bad arguments");
  if (int rc_ = enter(e)) return rc_;
  const int HW = e->g.HW, A = e->g.A;
  const int chunk = e->g.slots;
  std::vector<az::Board> hb(std::min(n, chunk));
  uint8_t* dmask = reinterpret_cast<uint8_t*>(e->probs);  // slots*A floats >= slots*A bytes
  for (int off = 0; off < n; off += chunk) {
    const int m = std::min(chunk, n - off);
    for (int i = 0; i < m; ++i) hb[i] = board_from_cells(boards + (size_t)(off + i) * HW, HW);
    AZ_HIP(hipMemcpyAsync(e->dev_boards, hb.data(), m * sizeof(az::Board), hipMemcpyHostToDevice, e->stream));
    if (state) {
      az::launch_encode(e->dev_boards, nullptr, m, HW, e->x, e->stream);
      AZ_HIP(hipMemcpyAsync(state + (size_t)off * HW * 4, e->x, (size_t)m * HW * 4 * sizeof(float),
                            hipMemcpyDeviceToHost, e->stream));
    }
    if (mask) {
      az::launch_legal_mask(e->dev_boards, m, e->g, dmask, e->stream);
      AZ_HIP(hipMemcpyAsync(mask + (size_t)off * A, dmask, (size_t)m * A, hipMemcpyDeviceToHost, e->stream));
    }
    AZ_HIP(hipStreamSynchronize(e->stream));
  }
  return 0;
}

int az_forward(az_engine* e, const float* x, int n, float* probs, float* values) {
  if (!e || n < 0 || (n && (!x || !probs || !values))) return fail(AZ_E_INVALID, "bad arguments");
  if (!e->net.ready) return fail(AZ_E_STATE, "az_engine_set_weights was not called");
  if (int rc_ = enter(e)) return rc_;
  const int HW = e->g.HW, A = e->g.A, chunk = e->g.slots;
  for (int off = 0; off < n; off += chunk) {
    const int m = std::min(chunk, n - off);
    AZ_HIP(hipMemcpyAsync(e->x, x + (size_t)off * HW * 4, (size_t)m * HW * 4 * sizeof(float),
                          hipMemcpyHostToDevice, e->stream));
    az::launch_forward(e->net, e->x, nullptr, m, e->g.H, e->g.W, A, e->act[0], e->act[1], e->act[2],
                       e->probs, e->values, e->stream, e->timer.enabled ? &e->timer : nullptr);
    AZ_HIP(hipGetLastError());
    AZ_HIP(hipMemcpyAsync(probs + (size_t)off * A, e->probs, (size_t)m * A * sizeof(float),
                          hipMemcpyDeviceToHost, e->stream));
    AZ_HIP(hipMemcpyAsync(values + off, e->values, (size_t)m * sizeof(float), hipMemcpyDeviceToHost,
                          e->stream));
    AZ_HIP(hipStreamSynchronize(e->stream));
  }
  return 0;
}

int az_stats_get(az_engine* e, az_stats* st) {
  if (!e || !st) return fail(AZ_E_INVALID, "null argument");
  AZ_HIP(hipSetDevice(e->device));
  int rc;
  if ((rc = sync_all(e))) return rc;
  unsigned long long h[az::kStatCount];
  AZ_HIP(hipMemcpy(h, e->t.stats, sizeof(h), hipMemcpyDeviceToHost));
  std::vector<int64_t> gid(e->g.slots);
  AZ_HIP(hipMemcpy(gid.data(), e->t.game_id, gid.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
  memset(st, 0, sizeof(*st));
  st->expansions = (int64_t)h[az::kStatExpansions];
  st->terminal_visits = (int64_t)h[az::kStatTerminal];
  st->games_done = (int64_t)h[az::kStatGamesDone];
  st->simulations = (int64_t)h[az::kStatSims];
  st->plies = (int64_t)h[az::kStatPlies];
  st->errors = (int64_t)h[az::kStatErrors];
  st->active_slots = std::count_if(gid.begin(), gid.end(), [](int64_t v) { return v >= 0; });
  std::vector<az::ConvTimer*> timers = {&e->timer, &e->whole.timer};
  for (Lane* L : e->lanes)
    if (L != &e->whole) timers.push_back(&L->timer);
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
  std::vector<az::ConvTimer*> ttimers = {&e->whole.tree_timer};
  for (Lane* L : e->lanes)
    if (L != &e->whole) ttimers.push_back(&L->tree_timer);
  for (az::ConvTimer* tm : ttimers) {
    tm->flush();
    st->tree_ms += tm->total_ms;
    st->tree_launches += tm->launches;
  }
  st->path_edges = (int64_t)h[az::kStatPathEdges];
  st->max_retained = (int64_t)h[az::kStatMaxRetained];
  st->cache_hits = (int64_t)h[az::kStatCacheHits];
  st->evaluations = (int64_t)h[az::kStatNNEvals];
  if (e->cache.ctl) {
    unsigned long long ctl[3];
    AZ_HIP(hipMemcpy(ctl, e->cache.ctl, sizeof(ctl), hipMemcpyDeviceToHost));
    st->cache_generation = (int64_t)ctl[0];
    st->cache_inserts = (int64_t)ctl[1];
    st->cache_gen_size = (int64_t)e->cache.gen_size;
    st->cache_entries = (int64_t)ctl[2];
    st->cache_capacity = (int64_t)e->cache.mask + 1;
  }
  st->games_drained = e->drained;
  st->arena_edges = e->g.arena_cap;
  if (e->g.halves > 1) {
    st->arena_pool_edges = 0;
    for (Lane* L : e->lanes) st->arena_pool_edges += 2 * L->pool_cap;
    st->arena_pool_high = (int64_t)h[az::kStatPoolHigh];
  }
  st->issued_flop_per_board = e->net.issued_flop_per_board;
  st->issued_flop_per_board_small = e->net.issued_flop_per_board_small;
  st->tower_small_max_boards = e->net.tower_small_max_boards;
  return 0;
}

int az_cache_enable(az_engine* e, int on) {
  if (!e) return fail(AZ_E_INVALID, "null engine");
  if (!e->cache.state) return on ? fail(AZ_E_STATE, "engine created with cache_log2 = 0") : 0;
  int rc;
  if ((rc = sync_all(e))) return rc;
  e->cache.enabled = on != 0;
  return 0;
}

int az_cache_clear(az_engine* e) {
  if (!e) return fail(AZ_E_INVALID, "null engine");
  AZ_HIP(hipSetDevice(e->device));
  return cache_clear(e);
}

int az_timer_enable(az_engine* e, int on) {
  if (!e) return fail(AZ_E_INVALID, "null engine");
  int rc;
  if ((rc = sync_all(e))) return rc;
  if (!e->timer_ref) AZ_HIP(hipEventCreate(&e->timer_ref));
  AZ_HIP(hipEventRecord(e->timer_ref, e->stream));
  AZ_HIP(hipStreamSynchronize(e->stream));
  // on: 1 = conv launches, 2 = conv + select/expand launches (more events per
  // simulation: bench.py times the tree kernels in a window of their own),
  // k >= 3 = every k-th conv launch of each lane (sampled)
  std::vector<az::ConvTimer*> timers = {&e->timer, &e->whole.timer}, ttimers = {&e->whole.tree_timer};
  for (Lane* L : e->lanes)
    if (L != &e->whole) {
      timers.push_back(&L->timer);
      ttimers.push_back(&L->tree_timer);
    }
  for (az::ConvTimer* tm : timers) {
    tm->flush();
    tm->reset();
    tm->ref = &e->timer_ref;
    tm->enabled = on != 0;
    tm->stride = on >= 3 ? on : 1;
  }
  for (az::ConvTimer* tm : ttimers) {
    tm->flush();
    tm->reset();
    tm->ref = &e->timer_ref;
    tm->enabled = on >= 2;
  }
  return 0;
}

int az_pow_table(az_engine* e, double* out, int64_t n) {
  if (!e || !out || n < 0 || n > e->g.pow_len) return fail(AZ_E_INVALID, "bad arguments");
  AZ_HIP(hipMemcpy(out, e->t.powtab, n * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

// ------------------------------------------------------------------ self-play
int az_selfplay_begin(az_engine* e, int64_t first_game, int64_t n_games, uint32_t base_seed) {
  if (!e || n_games < 0 || first_game < 0) return fail(AZ_E_INVALID, "bad arguments");
  int rc;
  e->broken = false;  // every slot starts a fresh game
  if ((rc = ready_to_search(e))) return rc;
  AZ_HIP(hipSetDevice(e->device));
  if ((rc = sync_all(e))) return rc;  // moves of an earlier batch may still be running (async steps)
  for (void* p : e->sample_bufs) (void)hipFree(p);
  e->sample_bufs.clear();
  az::SampleDev& smp = e->smp;
  smp = az::SampleDev{};
  smp.first_game = first_game;
  smp.n_games = n_games;
  smp.base_seed = base_seed;
  const size_t G = (size_t)std::max<int64_t>(n_games, 1), P = (size_t)e->g.HW, A = (size_t)e->g.A;
  auto get = [&](void** p, size_t bytes) -> int {
    AZ_HIP(hipMalloc(p, std::max<size_t>(bytes, 16)));
    e->sample_bufs.push_back(*p);
    AZ_HIP(hipMemsetAsync(*p, 0, std::max<size_t>(bytes, 16), e->stream));
    return 0;
  };
  if ((rc = get((void**)&smp.boards, G * P * sizeof(az::Board))) ||
      (rc = get((void**)&smp.policy, G * P * A * sizeof(double))) ||
      (rc = get((void**)&smp.moves, G * P * sizeof(int16_t))) ||
      (rc = get((void**)&smp.length, G * sizeof(int32_t))) ||
      (rc = get((void**)&smp.result, G * sizeof(int32_t))) ||
      (rc = get((void**)&smp.expansions, G * sizeof(int32_t))) ||
      (rc = get((void**)&smp.done_ids, G * sizeof(int64_t))) ||
      (rc = get((void**)&smp.done_count, sizeof(unsigned long long))))
    return rc;
  e->drained = 0;
  e->batch_first_move = e->moves_issued;
  unsigned long long st[az::kStatCount] = {0};
  const int64_t first_wave = std::min<int64_t>(n_games, e->g.slots);
  st[az::kStatNextGame] = (unsigned long long)(first_game + first_wave);
  AZ_HIP(hipMemcpyAsync(e->t.stats, st, sizeof(st), hipMemcpyHostToDevice, e->stream));
  az::launch_slot_init(e->g, e->t, smp, first_wave, e->stream);
  AZ_HIP(hipGetLastError());
  if (e->g.halves > 1)  // every slot starts with no chunk: the pools are empty
    for (Lane* L : e->lanes) {
      AZ_HIP(hipMemsetAsync(L->t.pool_top, 0, sizeof(unsigned long long), e->stream));
      AZ_HIP(hipMemsetAsync(L->t.dst_top, 0, sizeof(unsigned long long), e->stream));
    }
  AZ_HIP(hipStreamSynchronize(e->stream));
  e->sp_first = first_game;
  e->sp_n = n_games;
  return 0;
}

int az_selfplay_step(az_engine* e, int n_moves, az_stats* st) {
  if (!e || n_moves < 0) return fail(AZ_E_INVALID, "bad arguments");
  int rc;
  if ((rc = ready_to_search(e))) return rc;
  AZ_HIP(hipSetDevice(e->device));
  const bool multi = e->lanes.size() > 1;
  for (int mv = 0; mv < n_moves; ++mv) {
    const int64_t m = e->moves_issued++;
    // lanes interleaved per simulation so every stream always has work queued
    for (int s = 0; s < e->g.sims; ++s)
      for (Lane* L : e->lanes)
        if ((rc = simulate(e, *L))) return rc;
    for (Lane* L : e->lanes) {
      // a lane plays move m once every other lane has finished move m - 1, so
      // move m - 1's snapshot (taken by the last of them) holds no game of
      // move m; it also keeps the lanes within two moves of each other (the
      // cache eviction bound, az_tree.h)
      if (multi && m > e->batch_first_move)
        for (Lane* O : e->lanes)
          if (O != L) AZ_HIP(hipStreamWaitEvent(L->stream, O->move_done[(m - 1) % 4], 0));
      az::launch_play(L->g, L->t, e->smp, nullptr, -1, 0, 1, L->stream);
      az::launch_compact(L->g, L->t, L->stream);
      if (L->g.halves > 1) {  // the kept trees are in the other half now: it is the current one
        std::swap(L->t.edges, L->t.dst_edges);
        std::swap(L->t.pool_top, L->t.dst_top);
      }
      az::launch_move_end(e->move_arrive + m % 4, (int)e->lanes.size(), e->smp.done_count,
                          e->snap_dev + m % 4, L->stream);
      AZ_HIP(hipEventRecord(L->move_done[m % 4], L->stream));
    }
    AZ_HIP(hipGetLastError());
  }
  if (!st) return 0;  // asynchronous: the moves run on while the caller drains earlier ones
  if ((rc = sync_all(e))) return rc;
  if ((rc = check_device_errors(e))) return rc;
  return az_stats_get(e, st);
}

int az_selfplay_run(az_engine* e, int64_t first_game, int64_t n_games, uint32_t base_seed,
                    az_stats* st) {
  int rc;
  if ((rc = az_selfplay_begin(e, first_game, n_games, base_seed))) return rc;
  az_stats tmp;
  for (;;) {
    if ((rc = az_selfplay_step(e, 1, &tmp))) return rc;
    if (tmp.active_slots == 0) break;
  }
  if (st) *st = tmp;
  return 0;
}

int az_selfplay_results(az_engine* e, int32_t* lengths, int32_t* results, int32_t* expansions,
                        int8_t* boards, double* policies, int32_t* moves) {
  if (!e) return fail(AZ_E_INVALID, "null engine");
  if (int rc_ = enter(e)) return rc_;
  AZ_HIP(hipStreamSynchronize(e->stream));
  const size_t G = (size_t)e->sp_n, P = (size_t)e->g.HW, A = (size_t)e->g.A, HW = (size_t)e->g.HW;
  if (G == 0) return 0;
  const az::SampleDev& smp = e->smp;
  if (lengths) AZ_HIP(hipMemcpy(lengths, smp.length, G * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (results) AZ_HIP(hipMemcpy(results, smp.result, G * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (expansions) AZ_HIP(hipMemcpy(expansions, smp.expansions, G * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (policies) AZ_HIP(hipMemcpy(policies, smp.policy, G * P * A * sizeof(double), hipMemcpyDeviceToHost));
  if (boards) {
    std::vector<az::Board> hb(G * P);
    AZ_HIP(hipMemcpy(hb.data(), smp.boards, hb.size() * sizeof(az::Board), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < hb.size(); ++i) cells_from_board(hb[i], (int)HW, boards + i * HW);
  }
  if (moves) {
    std::vector<int16_t> hm(G * P);
    AZ_HIP(hipMemcpy(hm.data(), smp.moves, hm.size() * sizeof(int16_t), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < hm.size(); ++i) moves[i] = hm[i];
  }
  return 0;
}

int az_selfplay_drain(az_engine* e, int64_t max_games, int64_t* n_out, int64_t* game_ids, int32_t* lengths,
                      int32_t* results, int32_t* expansions, int8_t* boards, double* policies,
                      int32_t* moves) {
  if (!e || !n_out || max_games < 0) return fail(AZ_E_INVALID, "bad arguments");
  *n_out = 0;
  if (!e->smp.done_count) return 0;  // no self-play batch begun
  AZ_HIP(hipSetDevice(e->device));
  // the newest move whose count snapshot is complete; if the last issued
  // move is still running, wait for the one before it (never for the running one)
  // (a move's snapshot is complete once every lane has finished the move)
  const int64_t last = e->moves_issued - 1;
  int64_t k = -1;
  bool last_done = last >= e->batch_first_move;
  if (last_done)
    for (Lane* L : e->lanes) last_done = last_done && hipEventQuery(L->move_done[last % 4]) == hipSuccess;
  if (last_done) {
    k = last;
  } else if (last - 1 >= e->batch_first_move) {
    k = last - 1;
    for (Lane* L : e->lanes) AZ_HIP(hipEventSynchronize(L->move_done[k % 4]));
  }
  if (k < 0) return 0;
  const unsigned long long done = __atomic_load_n(e->snap_host + k % 4, __ATOMIC_ACQUIRE);
  const int64_t n = std::min<int64_t>((int64_t)done - e->drained, max_games);
  if (n <= 0) return 0;
  const size_t rec = az::drain_record_bytes(e->g);
  if ((size_t)n > e->drain_cap) {
    if (e->drain_dev) AZ_HIP(hipFree(e->drain_dev));
    if (e->drain_host) AZ_HIP(hipHostFree(e->drain_host));
    e->drain_dev = nullptr;
    e->drain_host = nullptr;
    e->drain_cap = 0;
    const size_t cap = std::max<size_t>((size_t)n, 1024);
    AZ_HIP(hipMalloc(&e->drain_dev, cap * rec));
    AZ_HIP(hipHostMalloc(&e->drain_host, cap * rec, hipHostMallocDefault));
    e->drain_cap = cap;
  }
  // pack_stream (nothing else queued on it; the host has seen move k finish
  // on every lane): games up to move k are complete
  az::launch_drain_pack(e->g, e->smp, e->drained, (int)n, e->drain_dev, e->pack_stream);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipMemcpyAsync(e->drain_host, e->drain_dev, (size_t)n * rec, hipMemcpyDeviceToHost, e->pack_stream));
  AZ_HIP(hipStreamSynchronize(e->pack_stream));
  const size_t HW = (size_t)e->g.HW, A = (size_t)e->g.A;
  for (int64_t i = 0; i < n; ++i) {
    const uint8_t* r = e->drain_host + (size_t)i * rec;
    const int32_t* h = reinterpret_cast<const int32_t*>(r + 8);
    if (game_ids) memcpy(game_ids + i, r, sizeof(int64_t));
    if (lengths) lengths[i] = h[0];
    if (results) results[i] = h[1];
    if (expansions) expansions[i] = h[2];
    if (policies) memcpy(policies + i * HW * A, r + 24, HW * A * sizeof(double));
    const int16_t* mv = reinterpret_cast<const int16_t*>(r + 24 + 8 * HW * A);
    if (moves)
      for (size_t p = 0; p < HW; ++p) moves[i * HW + p] = mv[p];
    if (boards) memcpy(boards + i * HW * HW, mv + HW, HW * HW);
  }
  e->drained += n;
  *n_out = n;
  return 0;
}

// ------------------------------------------------------------------ tree API
int az_tree_reset(az_engine* e, int n, const int32_t* slots, const int8_t* boards) {
  if (!e || n < 0 || n > e->g.slots || (n && (!slots || !boards))) return fail(AZ_E_INVALID, "bad arguments");
  if (int rc_ = enter(e)) return rc_;
  if (int rc_ = tree_api_ok(e)) return rc_;
  std::vector<az::Board> hb(n);
  for (int i = 0; i < n; ++i) {
    if (slots[i] < 0 || slots[i] >= e->g.slots) return fail(AZ_E_INVALID, "slot out of range");
    hb[i] = board_from_cells(boards + (size_t)i * e->g.HW, e->g.HW);
  }
  e->smp = az::SampleDev{};
  AZ_HIP(hipMemcpyAsync(e->dev_i32, slots, n * sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
  AZ_HIP(hipMemcpyAsync(e->dev_boards, hb.data(), n * sizeof(az::Board), hipMemcpyHostToDevice, e->stream));
  az::launch_slot_set_root(e->g, e->t, e->dev_i32, e->dev_boards, n, e->stream);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipStreamSynchronize(e->stream));
  e->broken = false;
  return 0;
}

int az_tree_release(az_engine* e, int n, const int32_t* slots) {
  if (!e || n < 0 || n > e->g.slots || (n && !slots)) return fail(AZ_E_INVALID, "bad arguments");
  if (int rc_ = enter(e)) return rc_;
  for (int i = 0; i < n; ++i)
    if (slots[i] < 0 || slots[i] >= e->g.slots) return fail(AZ_E_INVALID, "slot out of range");
  AZ_HIP(hipMemcpyAsync(e->dev_i32, slots, n * sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
  az::launch_slot_release(e->t, e->dev_i32, n, e->stream);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipStreamSynchronize(e->stream));
  return 0;
}

int az_tree_search(az_engine* e, int n_sims) {
  if (!e || n_sims < 0) return fail(AZ_E_INVALID, "bad arguments");
  if (e->g.noise)  // the tree API's noise is drawn by the caller from numpy's global stream
    return fail(AZ_E_INVALID, "this engine mixes Dirichlet root noise: search it with az_tree_search_noise "
                              "(the caller's np.random.dirichlet draws)");
  int rc;
  if ((rc = ready_to_search(e))) return rc;
  if (int rc_ = enter(e)) return rc_;
  if (int rc_ = tree_api_ok(e)) return rc_;
  for (int s = 0; s < n_sims; ++s)
    if ((rc = simulate(e, e->whole))) return rc;
  AZ_HIP(hipStreamSynchronize(e->stream));
  return check_device_errors(e);
}

int az_tree_search_noise(az_engine* e, int n_sims, const double* noise, int rows) {
  if (!e || n_sims < 0 || rows < 0 || (rows > 0 && !noise)) return fail(AZ_E_INVALID, "bad arguments");
  if (!e->g.noise)
    return fail(AZ_E_INVALID, "az_tree_search_noise needs an engine created with dirichlet_noise = 1");
  int rc;
  if ((rc = ready_to_search(e))) return rc;
  if (int rc_ = enter(e)) return rc_;
  if (int rc_ = tree_api_ok(e)) return rc_;
  const size_t S = (size_t)e->g.slots, n = S * (size_t)std::max(rows, 1) * e->g.A;
  az::TreeDev& t = e->whole.t;
  if (n > e->noise_cap) {  // grown on demand, kept for the next searches
    double* buf = nullptr;
    if ((rc = e->alloc(&buf, n))) return rc;
    e->noise_buf = buf;
    e->noise_cap = n;
  }
  if (!t.noise_cur && (rc = e->alloc(&t.noise_cur, S))) return rc;
  if (rows) AZ_HIP(hipMemcpyAsync(e->noise_buf, noise, S * rows * e->g.A * sizeof(double), hipMemcpyHostToDevice,
                                  e->stream));
  AZ_HIP(hipMemsetAsync(t.noise_cur, 0, S * sizeof(int32_t), e->stream));
  t.noise_in = e->noise_buf;
  t.noise_rows = rows;
  rc = 0;
  for (int s = 0; s < n_sims && !rc; ++s) rc = simulate(e, e->whole);
  t.noise_in = nullptr;  // self-play keeps drawing on the device
  t.noise_rows = 0;
  if (rc) return rc;
  AZ_HIP(hipStreamSynchronize(e->stream));
  return check_device_errors(e);
}

int az_tree_play(az_engine* e, const double* uniforms, int greedy, int deterministic,
                 int32_t* moves, int32_t* status, double* policy) {
  if (!e || (!deterministic && !uniforms)) return fail(AZ_E_INVALID, "bad arguments");
  if (e->broken) return ready_to_search(e);
  if (int rc_ = enter(e)) return rc_;
  if (int rc_ = tree_api_ok(e)) return rc_;
  const size_t S = (size_t)e->g.slots;
  if (!deterministic)
    AZ_HIP(hipMemcpyAsync(e->uniforms, uniforms, S * sizeof(double), hipMemcpyHostToDevice, e->stream));
  AZ_HIP(hipMemsetAsync(e->t.last_move, 0xff, S * sizeof(int32_t), e->stream));
  az::SampleDev none{};
  az::launch_play(e->g, e->t, none, deterministic ? nullptr : e->uniforms, greedy ? 1 : 0,
                  deterministic, 0, e->stream);
  AZ_HIP(hipGetLastError());
  if (moves) AZ_HIP(hipMemcpyAsync(moves, e->t.last_move, S * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  if (status) AZ_HIP(hipMemcpyAsync(status, e->t.last_status, S * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  if (policy)
    AZ_HIP(hipMemcpyAsync(policy, e->t.last_policy, S * e->g.A * sizeof(double), hipMemcpyDeviceToHost, e->stream));
  AZ_HIP(hipStreamSynchronize(e->stream));
  return check_device_errors(e);
}

int az_tree_info(az_engine* e, int slot, int64_t* info, float* root_value) {
  if (!e || !info || slot < 0 || slot >= e->g.slots) return fail(AZ_E_INVALID, "bad arguments");
  if (int rc_ = enter(e)) return rc_;
  AZ_HIP(hipStreamSynchronize(e->stream));
  int32_t top, first, cnt, ply;
  int64_t gid;
  AZ_HIP(hipMemcpy(&top, e->t.arena_top + slot, 4, hipMemcpyDeviceToHost));
  AZ_HIP(hipMemcpy(&first, e->t.root_first + slot, 4, hipMemcpyDeviceToHost));
  AZ_HIP(hipMemcpy(&cnt, e->t.root_n + slot, 4, hipMemcpyDeviceToHost));
  AZ_HIP(hipMemcpy(&ply, e->t.ply + slot, 4, hipMemcpyDeviceToHost));
  AZ_HIP(hipMemcpy(&gid, e->t.game_id + slot, 8, hipMemcpyDeviceToHost));
  if (root_value) AZ_HIP(hipMemcpy(root_value, e->t.root_value + slot, 4, hipMemcpyDeviceToHost));
  info[0] = top;
  info[1] = first;
  info[2] = cnt;
  info[3] = ply;
  info[4] = gid >= 0;
  return 0;
}

int az_tree_export(az_engine* e, int slot, double* prior, double* w, int32_t* n, int32_t* child,
                   int32_t* child_n, int32_t* action, float* child_value) {
  if (!e || slot < 0 || slot >= e->g.slots) return fail(AZ_E_INVALID, "bad arguments");
  if (int rc_ = enter(e)) return rc_;
  AZ_HIP(hipStreamSynchronize(e->stream));
  if (int rc_ = tree_api_ok(e)) return rc_;
  int32_t top;
  AZ_HIP(hipMemcpy(&top, e->t.arena_top + slot, 4, hipMemcpyDeviceToHost));
  std::vector<az::Edge> h(top);
  if (top)
    AZ_HIP(hipMemcpy(h.data(), e->t.edges + (size_t)slot * e->g.arena_cap, top * sizeof(az::Edge),
                     hipMemcpyDeviceToHost));
  for (int i = 0; i < top; ++i) {
    if (prior) prior[i] = h[i].prior;
    if (w) w[i] = h[i].W;
    if (n) n[i] = h[i].N;
    if (child) child[i] = h[i].child;
    if (child_n) child_n[i] = h[i].child_n;
    if (action) action[i] = h[i].action & az::kActMask;
    if (child_value) child_value[i] = h[i].child_value;
  }
  return 0;
}

}  // extern "C"
