// az_nn.h -- device-side network weights and the forward launchers.
#pragma once
#include <vector>

#include "../../include/az.h"
#include "az_device.h"

namespace az {

// tower16_kernel (az_tower16.hip): the whole Connect-N forward in one launch.
// Its view of the network, resident in device memory (kernel reads it with
// scalar loads).
constexpr int kTowerMaxDepth = 16;   // residual blocks
constexpr int kTowerMaxBoards = 8;   // boards per workgroup tile
struct TowerNet {
  const uint4* k1[kTowerMaxDepth];   // conv16 packs: conv1 (36 k-steps)
  const uint4* k2[kTowerMaxDepth];   // conv2 + 1x1 projection residual (40)
  float s1[kTowerMaxDepth];          // 2^(e - 12) of each pack's prescale e
  float s2[kTowerMaxDepth];
  const uint4* stem16;               // the stem as 2 k-steps over k = tap*4 + plane (tower16_stem_pack)
  float stem_s;                      // its 2^(e - 12)
  const uint4* stem_k;               // input-row stem (chess, 118 planes padded to F): a conv16 pack, 36 k-steps
  float stem_ks;                     // its 2^(e - 12)
  // small weights, one contiguous float blob; a prefix of it is copied into
  // LDS at kernel start (offsets in floats, each a multiple of 4): folded
  // biases b1[depth][F], b2[depth][F] (+ the residual's), stem bias [F]; head
  // 1x1 convs wpc [F][2], wvc [F], hb = {bpc0, bpc1, bvc0, bv2}; policy bias
  // bpd [A]; value dense bv1 [hidden], wv2 [hidden]; then the two large
  // matrices, staged only when the LDS holds them (else read from L2):
  // policy dense wpd [2HW][A] (wpd_lds), value dense wv1 [HW][hidden] (wv1_lds)
  const float* blob;
  int blob_floats, staged_floats;    // whole blob; the prefix staged in LDS
  int off_b1, off_b2, off_stemb, off_wpc, off_wvc, off_hb, off_bpd, off_bv1, off_wv2, off_wpd, off_wv1;
  int wpd_lds, wv1_lds;
  int wv1_xtile;                     // not staged, but DMA'd behind the heads' partials in X's tile (dbuf)
  int dbuf;                          // two activation tiles (else one, updated in place)
  int depth, hidden;
  int tile_rows;                     // 96, 128 or 256 pixel rows per workgroup tile
  // slot plan (tower16_slot_plan; null: natural order, no skips): the pixel
  // word of each of a full tile's slots, and per M half the blocks each tap
  // skips (2 bits per tap over the wave's blocks 0 and 1)
  const int* slot_pix;
  int skip[2];
  // dual launches (tower16_dual_kernel): an alternative, shorter tile height
  // for launches of at most alt_max_boards live boards, with its own slot
  // plan (0 / null: one tile height)
  int alt_rows;
  const int* alt_slot_pix;
  int alt_skip[2];
  int alt_max_boards;
  // its LDS staging: the blob prefix (the 96-row layout holds the whole blob,
  // value dense wv1 included, where the 128-row one leaves wv1 in L2)
  int alt_staged_floats, alt_wpd_lds, alt_wv1_lds;
};
// the slot plan of 128-row tiles: border blocks (16 slots whose pixels all
// sit on one board edge) skip the three taps that read past that edge; empty
// vectors when no plan applies (then natural order)
void tower16_slot_plan(int H, int W, int tile_rows, std::vector<int>& slot_pix, int skip[2]);
// MFMA FLOP tower16_kernel issues per board: a full tile's stem + 2 depth
// convs (+ the 1x1 projection k-steps) less the plan's skipped taps, / boards
// (rows_stem: the input-row stem, stem_chunks of its 4 input chunks computed)
double tower16_issued_flop_per_board(int HW, int tile_rows, int depth, const int skip[2], bool rows_stem = false,
                                     int stem_chunks = 4);
// 0 when the board does not fit a tile (HW > 128); else 96 or 128 (big:
// 256-row tiles, 16 M blocks, each wave 128 rows x 32 channels -- half the
// weight stream per FLOP; single tile in place, the LDS holds no second)
int tower16_tile_rows(int HW);
int tower16_boards_per_tile(int HW, int tile_rows);
// LDS of one workgroup: activation rows (one or two tiles + zero rows) +
// bookkeeping + staged blob floats
size_t tower16_lds_bytes(int HW, int tile_rows, int staged_floats, bool dbuf);
// whether the heads' scratch (features, logits, partials) fits the tiles
bool tower16_heads_fit(int HW, int tile_rows, int A, int hidden, bool dbuf);
// whether wv1 [HW][hidden] fits X's tile behind the heads' partials (dbuf)
bool tower16_wv1_xtile_fits(int HW, int tile_rows, int hidden);
constexpr size_t kTowerLdsMax = 160 * 1024;
// host: folded stem [3][3][4][F] (Keras order) -> the stem16 pack with prescale e
void tower16_stem_pack(const double* w, int e, std::vector<uint16_t>& out);
// boards (self-play: the eval queue's boards) or x ([n][HW][4] one-hot planes,
// az_forward) -> probs [n][A], values [n]; count (device, may be null -> n_max)
// alt_rows: the TowerNet's alternative tile height (a dual launch), 0 = none
void launch_tower16(const TowerNet* net, int tile_rows, int alt_rows, int alt_staged_floats, int staged_floats,
                    bool dbuf, const Board* boards,
                    const float4* x, const int* count, int n_max, int H, int W, int A, float* probs, float* values,
                    unsigned long long* err, hipStream_t s);
// the input-row form (chess): rows [n][HW] of 512 B split16 (t0 of F
// channels, t1 x 2^12; az_nn's store_act4) -> the stem, the residual tower
// and the heads' 1x1 convs; per pixel float4 (relu(p0), relu(p1), relu(v), 0)
// into feat [n * HW] for the dense heads' kernels (policy_dense_kernel,
// heads_tail_kernel).  first_chunk: input channel chunks (32) below it are
// known zero and skipped (chess self-play: planes 0-63)
// chess self-play (round 5): the tower builds its boards' input planes in
// LDS from the leaves the select launch queued -- queue entry b's slot
// eval_slot[b], its position leaf[slot] (az_chess_pos), path_len / initial
// for the history form -- instead of reading rows an encode launch wrote
// (the same bits: az_chess.h full_state4 is encode_queue_kernel's code)
struct TowerLeaves {
  const int32_t* eval_slot = nullptr;
  const void* leaf = nullptr;
  const int32_t* path_len = nullptr;
  const int32_t* initial = nullptr;
};
void launch_tower16_rows(const TowerNet* net, int tile_rows, int staged_floats, bool dbuf, const void* rows,
                         int first_chunk, const int* count, int n_max, int H, int W, float4* feat,
                         unsigned long long* err, hipStream_t s, const TowerLeaves* leaves = nullptr);

// Folded (BatchNorm-in) weights resident in HBM, packed for the kernels (not
// Keras layouts).  AZ_CONV_F16X2 (default): conv16_kernel packs (fp16 term
// pairs, az_conv16.hip) and split16 activations; AZ_CONV_DIRECT: fp32 MFMA
// fragment packs ([chunk][tile][q][lane] float4) and fp32 activations.
struct NetDev {
  int filters = 128, depth = 0, hidden = 256;
  int algo = 0;             // AZ_CONV_F16X2 / AZ_CONV_DIRECT (one algorithm for every forward)
  bool use_tower = false;   // Connect-N, AZ_CONV_F16X2: the whole forward in tower16_kernel (else per layer)
  bool tower_natural_order = false;  // az_config.tower_natural_order: no slot plan (A/B, bitwise the same)
  TowerNet* tower = nullptr;  // device copy of the tower's view (load_network)
  int tower_staged = 0;       // its blob floats staged in LDS
  bool tower_dbuf = false;    // its activations double-buffered (TowerNet::dbuf)
  int tower_rows = 0;         // its tile rows (TowerNet::tile_rows)
  int tower_alt_staged = 0;   // its staged blob floats (TowerNet::alt_staged_floats)
  int tower_alt_rows = 0;     // the dual launch's alternative tile rows (TowerNet::alt_rows; 0 none)
  int lanes = 1;              // the engine's lanes (streams whose towers share the CUs): the dual threshold
  int in_ch = 4;            // input planes: 4 (Connect-N) or 118 (chess, padded to F)
  int board_h = 0, board_w = 0;  // Connect-N board (the tower's slot plan)
  double issued_flop_per_board_small = 0;  // the dual launch's alternative tiles (az_stats)
  int tower_small_max_boards = -1;          // TowerNet::alt_max_boards (az_stats)
  double issued_flop_per_board = 0;  // MFMA FLOP a forward issues per board (tower; az_stats)
  float* stem_w = nullptr;  // in_ch == 4: [36][F] (k = tap*4 + c), VALU stem kernels
  float* stem_b = nullptr;  // [F]
  // in_ch > 4 (chess): the stem is one more 3x3 conv over the zero-padded planes
  uint16_t* stem_k = nullptr;  // conv16 pack (36 k-steps)
  float stem_scale = 1.f;      // its 2^(e-12)
  float* stem_d = nullptr;     // direct-kernel fragments [9F x F]
  std::vector<uint16_t*> k1, k2;  // conv16 packs: conv1 (36 k-steps), conv2 + 1x1 residual (40)
  std::vector<float> k1_scale, k2_scale;
  std::vector<float*> c1_w, c1_b;  // direct: fragment-packed [9F x F]; folded bias [F]
  std::vector<float*> c2_w, c2_b;  // direct: [10F x F] (conv2 taps, then the 1x1 residual); bias conv2 + res
  float *pc_w = nullptr, *pc_b = nullptr;  // policy conv [F][2], [2]
  float *vc_w = nullptr, *vc_b = nullptr;  // value conv [F], [1]
  float *pd_w = nullptr, *pd_b = nullptr;  // policy dense [2HW][A], [A]
  float* pd_wt = nullptr;  // A > kMaxActions (chess): [ceil(A/64)][2HW][64], one contiguous slab per
                           // policy_dense_kernel column tile, zero past A
  float *v1_w = nullptr, *v1_b = nullptr;  // value dense1 [HW][hidden], [hidden]
  float *v2_w = nullptr, *v2_b = nullptr;  // value dense2 [hidden], [1]
  unsigned long long* err = nullptr;       // the engine's device error word (kErrActRange)
  bool ready = false;
};

// hipEvent pairs around the conv launches of every forward while enabled, so
// bench.py can price the dominant kernel live (roofline.achieved).  `ref` is
// an event the engine records when timing starts: intervals of all lanes are
// placed on one device clock, so their union (time in which any conv ran)
// can be taken next to the summed durations.
struct ConvTimer {
  bool enabled = false;
  // every stride-th launch timed (1: all): each event pair is a marker packet
  // on the lane's stream between the kernels it brackets, on the simulation
  // chain (bench.py's window: 1.2% of games/s with every launch timed,
  // profiles/r6/ab_exp5.txt)
  int stride = 1;
  long long seq = 0;
  bool cur = false;
  hipEvent_t* ref = nullptr;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  double total_ms = 0.0;
  long long launches = 0;
  std::vector<std::pair<double, double>> intervals;  // [start, end) ms after *ref
  void begin(hipStream_t s) {
    if (!enabled) return;
    cur = seq++ % stride == 0;
    if (!cur) return;
    if (used + 2 > pool.size()) {
      for (int i = 0; i < 256; ++i) {
        hipEvent_t e;
        // timing only: no system-scope fence (a default event's cache
        // writeback/invalidate cost ~12 us between the kernels it sits between)
        (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
        pool.push_back(e);
      }
    }
    (void)hipEventRecord(pool[used++], s);
  }
  void end(hipStream_t s, int n_launches) {
    if (!enabled || !cur) return;
    (void)hipEventRecord(pool[used++], s);
    launches += n_launches;
  }
  // call after a stream synchronize: folds recorded pairs into total_ms
  void flush() {
    for (size_t i = 0; i + 1 < used; i += 2) {
      float ms = 0.f, a = 0.f, b = 0.f;
      (void)hipEventElapsedTime(&ms, pool[i], pool[i + 1]);
      total_ms += ms;
      if (ref && hipEventElapsedTime(&a, *ref, pool[i]) == hipSuccess &&
          hipEventElapsedTime(&b, *ref, pool[i + 1]) == hipSuccess)
        intervals.emplace_back(a, b);
    }
    used = 0;
  }
  void reset() {
    used = 0;
    total_ms = 0.0;
    launches = 0;
    seq = 0;
    intervals.clear();
  }
  ~ConvTimer() {
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

void launch_encode(const Board* boards, const int* count, int n_max, int HW, float* x,
                   hipStream_t s);
void launch_legal_mask(const Board* boards, int n, const GameCfg& g, uint8_t* mask,
                       hipStream_t s);
// conv16_kernel (az_conv16.hip): direct 3x3 conv on the fp16 MFMA with
// split16 activations (x ~= t0 + t1 * 2^-12, per pixel 512 B: t0 of the 128
// channels, then t1) and host-packed two-term weights (conv16_pack)
struct Conv16Heads {
  const float* wpc;  // [F][2]
  const float* bpc;  // [2]
  const float* wvc;  // [F]
  const float* bvc;  // [1]
  float4* feat;      // non-null: the heads' 1x1 convs instead of storing the block output
};
struct Conv16Args {
  const void* in = nullptr;      // split16 rows [n_max*H*W]
  const void* res_in = nullptr;  // block input (fused 1x1 projection residual), or null
  const void* wpack = nullptr;   // conv16_pack layout (36 or 40 k-steps)
  const float* bias = nullptr;   // folded BN bias (+ the residual's)
  float oscale = 1.f;            // 2^(e - 12) for the weights' prescale e
  void* out = nullptr;           // split16 rows
  Conv16Heads heads{};
  const int* count = nullptr;    // live boards (device), or null -> n_max
  int n_max = 0, H = 0, W = 0;
  int mb = 4;                    // 16-row M blocks per workgroup tile (2, 3 or 4)
  int first_chunk = 0;           // 2: input channels 0..63 are known zero (chess self-play stem)
  unsigned long long* err = nullptr;  // device error word: kErrActRange if an output leaves the split16 range
};
void launch_conv16(const Conv16Args& a, hipStream_t s);
size_t conv16_lds_bytes(int MB, int W, bool res);
// power-of-two prescale e of a conv's weights (max |w * 2^-e| in (4, 8])
int conv16_prescale(const double* w, size_t n, const double* w2, size_t n2);
// weights [3][3][cin_n][128] (+ 1x1 residual [128][128]) -> uint16 fp16 bits
void conv16_pack(const double* w3, int cin_n, const double* wr, int e, std::vector<uint16_t>& out);
// Folds and uploads the network weights (Keras names, model/weights.py);
// device buffers are appended to `owned` (az_engine.hip)
int load_network(NetDev& net, const ::az_tensor* tensors, int n, int in_ch, int HW, int A,
                 double eps, std::vector<void*>& owned);
// x: [n][HW][4] fp32 (in_ch == 4), or the zero-padded planes [n][HW][F] (in_ch > 4) as split16 rows
// (AZ_CONV_F16X2) or fp32 (AZ_CONV_DIRECT); count (device int, may be null -> n_max) is the live
// batch; boards (optional): one-hot input straight from the eval queue's boards (bitwise the same
// outputs as encoding them into x first); stem_first_chunk: input planes below 32 * it are known zero
void launch_forward(const NetDev& net, const void* x, const int* count, int n_max, int H, int W,
                    int A, void* act_a, void* act_b, void* act_c, float* probs, float* values,
                    hipStream_t s, ConvTimer* timer, const Board* boards = nullptr,
                    int stem_first_chunk = 0, const TowerLeaves* leaves = nullptr);
// fp32 rows [n][c_src] -> the network's input layout for in_ch > 4: [n][F] zero-padded, as split16
// rows (split = true) or fp32
void launch_pad_rows(const float* src, int n, int c_src, void* dst, bool split, hipStream_t s);

// split16 of 8 floats: x ~= t0 + t1 * 2^-12 (t0 = fp16_rn(x), t1 = fp16_rn((x - t0) * 2^12), the
// subtraction exact), 8 fp16 each -- the layout every kernel writing conv16 input uses
typedef _Float16 az_h2 __attribute__((ext_vector_type(2)));
typedef float az_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_f16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((az_f2{a, b}), az_h2));
}
__device__ __forceinline__ void split16x8(const float (&x)[8], uint4& t0, uint4& t1) {
  uint32_t p[4], q[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p[i] = pk_f16(x[2 * i], x[2 * i + 1]);
    const az_h2 h = __builtin_bit_cast(az_h2, p[i]);
    q[i] = pk_f16((x[2 * i] - (float)h[0]) * 4096.f, (x[2 * i + 1] - (float)h[1]) * 4096.f);
  }
  t0 = make_uint4(p[0], p[1], p[2], p[3]);
  t1 = make_uint4(q[0], q[1], q[2], q[3]);
}
__device__ __forceinline__ void split16x4(const float4 v, uint2& t0, uint2& t1) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t p[2], q[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    p[i] = pk_f16(x[2 * i], x[2 * i + 1]);
    const az_h2 h = __builtin_bit_cast(az_h2, p[i]);
    q[i] = pk_f16((x[2 * i] - (float)h[0]) * 4096.f, (x[2 * i + 1] - (float)h[1]) * 4096.f);
  }
  t0 = make_uint2(p[0], p[1]);
  t1 = make_uint2(q[0], q[1]);
}
// store 4 channels (c4 = channel / 4) of an activation row: fp32 or split16
template <bool SPLIT>
__device__ __forceinline__ void store_act4(void* act, size_t row, int c4, const float4 v) {
  if constexpr (SPLIT) {
    uint2 t0, t1;
    split16x4(v, t0, t1);
    uint2* r = reinterpret_cast<uint2*>(reinterpret_cast<char*>(act) + row * 512);
    r[c4] = t0;
    r[32 + c4] = t1;
  } else {
    reinterpret_cast<float4*>(act)[row * 32 + c4] = v;
  }
}

}  // namespace az
