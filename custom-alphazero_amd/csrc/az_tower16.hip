// az_tower16.hip -- the whole Connect-N policy/value forward in ONE kernel
// (model/tensorflow/model.py:152-188 at inference): stem, the residual
// tower's 2*depth 3x3 convs, the heads' 1x1 convs, the dense layers, softmax
// and tanh.
//
// A workgroup owns WHOLE boards (Connect-4: 3 boards = 126 pixel rows of a
// 128-row tile) and keeps their activations in LDS from the stem to the
// heads.  A 3x3 'same' conv never reads outside its own board (off-board
// neighbours are the zero row), so a tile needs no halo, no layer's output
// makes an HBM round trip and a forward is one launch instead of eleven.
// Per-layer work is the split16 scheme of az_conv16.hip: activations
// x ~= t0 + t1 * 2^-12 and prescaled weights w' = b0 + b1 * 2^-12 as fp16
// term pairs, three v_mfma_f32_16x16x32_f16 per k-step into one fp32
// accumulator (t1*b0 + t0*b1 + t0*B0, B0 = 2^12 b0), so every layer is
// fp32-accurate (network error vs float64 ~1e-7).
//
// Workgroup = 8 waves (two per SIMD): wave w takes M half w >> 2 (MBW 16-row
// blocks) and N quarter w & 3 (32 output channels).  The weights are the
// MFMA's A operand, so a lane's accumulators are 4 consecutive channels of
// one pixel: an epilogue writes its split16 terms to LDS as 8-byte stores
// straight from the registers.  B fragments (host-packed, conv16_pack) stream
// from L2 into registers PF k-steps ahead; activation fragments are read from
// LDS one k-step ahead (the c16_phys rotation keeps every ds_read_b128 lane
// group on 16 distinct bank quads for any tap shift).
//
// The block's 1x1 projection residual (base_layers.py:95-125) is computed in
// conv1's phase (4 k-steps on the block input's own rows, into a second
// accumulator), because conv1's output then overwrites the block input in
// LDS; conv2 accumulates its taps on top of it.
//
// Range: a split16 term is fp16, so a stored activation must stay within
// +-32752.  Each board carries a power-of-two scale per activation buffer:
// a layer output whose board maximum exceeds the range is stored as
// y * 2^-s (s the smallest that fits) and the next conv multiplies its
// accumulator back by 2^s (exact).  The scale depends only on the board's
// own values, so results stay batch invariant; with no overflow (every
// network we have seen) s = 0 everywhere and nothing is rescaled.
//
// Every output element is summed in a fixed order (k-step, then term; heads
// in a fixed tree), so a board's outputs do not depend on its position in
// the tile or on the rest of the batch -- the oracle replay tests rely on it.
#include <algorithm>
#include <cmath>

#include "az_nn.h"
#include "az_tree.h"

namespace az {

typedef _Float16 t_h8 __attribute__((ext_vector_type(8)));
typedef float t_f4 __attribute__((ext_vector_type(4)));

namespace {

constexpr float kRange = 32752.f;  // largest |x| a split16 term pair holds
constexpr int kThreads = 512;

__device__ __forceinline__ int phys_slot(int x, int j) { return (j & 16) | ((j + 2 * x) & 15); }

__device__ __forceinline__ t_h8 unscale_b0(const uint4 v) {
  return __builtin_bit_cast(t_h8, v) * (_Float16)0.000244140625f;
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// smallest s >= 0 with m * 2^-s <= kRange (m >= 0, finite)
__device__ __forceinline__ int range_exp(float m) {
  int s = 0;
  while (ldexpf(m, -s) > kRange) ++s;
  return s;
}

// Shared bookkeeping after the activation rows.
struct TowerSmem {
  int flag[2];              // overflow seen in the layer being stored (alternating by layer)
  int sc[2][kTowerMaxBoards];  // per-board scale exponent of the two activation buffers' contents
  unsigned bmax[kTowerMaxBoards];  // board maxima (float bits, values >= 0) on the rare rescale path
  float vred[kTowerMaxBoards][4];  // value-head partial sums per board and wave
};

// store 4 channels (channel quad cq) of activation row r as split16 terms
__device__ __forceinline__ void put4(uint4* act, int r, int cq, const float4 y) {
  uint2 t0, t1;
  split16x4(y, t0, t1);
  char* row = reinterpret_cast<char*>(act) + (size_t)r * 512;
  const int j = cq >> 1, half = (cq & 1) * 8;
  *reinterpret_cast<uint2*>(row + phys_slot(r, j) * 16 + half) = t0;
  *reinterpret_cast<uint2*>(row + phys_slot(r, 16 + j) * 16 + half) = t1;
}

__device__ __forceinline__ float max4(const float4 v) { return fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)); }
__device__ __forceinline__ float4 scale4(const float4 v, float s) {
  return make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
}

// Store one layer's output (NI float4 items per thread: row, channel quad,
// board, value >= 0; row < 0 = no item).  Optimistic at scale 0; if any
// value left the split16 range, the boards concerned are stored again at
// their scale.  Returns whether any board of this buffer is scaled (then
// sc_out holds the exponents).  Contains the barrier that publishes the
// stores.  `par` alternates per layer (flag[par] is this layer's).
template <int NI>
__device__ __forceinline__ bool store_layer(uint4* act, const int (&row_)[NI], const int (&cq_)[NI], const int (&brd_)[NI],
                            const float4 (&y)[NI], TowerSmem& sm, int par, int* sc_out, int nbrd,
                            unsigned long long* err) {
  // rows, quads and boards laundered (as in k_loop): the addresses derived
  // from them are recomputed here, not hoisted out of the depth loop and spilled
  int row[NI], cq[NI], brd[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    row[i] = row_[i];
    cq[i] = cq_[i];
    brd[i] = brd_[i];
    asm volatile("" : "+v"(row[i]), "+v"(cq[i]), "+v"(brd[i]));
  }
  float vmax = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (row[i] >= 0) {
      vmax = fmaxf(vmax, max4(y[i]));
      put4(act, row[i], cq[i], y[i]);
    }
  if (!(vmax <= kRange)) sm.flag[par] = 1;  // also NaN
  if (threadIdx.x == 0) sm.flag[par ^ 1] = 0;  // next layer's flag (nobody reads it before then)
  __syncthreads();
  if (!sm.flag[par]) return false;  // workgroup-uniform
  // rare: board maxima, then the scaled boards' rows again
  if ((int)threadIdx.x < nbrd) sm.bmax[threadIdx.x] = 0u;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (row[i] >= 0) atomicMax(&sm.bmax[brd[i]], __float_as_uint(max4(y[i])));
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (row[i] < 0) continue;
    const float m = __uint_as_float(sm.bmax[brd[i]]);
    if (!(m <= 3.0e38f)) continue;  // inf/NaN: flagged below, nothing to rescale
    const int s = range_exp(m);
    if (s) put4(act, row[i], cq[i], scale4(y[i], ldexpf(1.f, -s)));
  }
  if ((int)threadIdx.x < nbrd) {
    const float m = __uint_as_float(sm.bmax[threadIdx.x]);
    if (!(m <= 3.0e38f)) {
      if (err) atomicOr(err, kErrActRange);
      sc_out[threadIdx.x] = 0;
    } else {
      sc_out[threadIdx.x] = range_exp(m);
    }
  }
  __syncthreads();
  return true;
}

// one k-step's 6*MBW MFMAs: weights as the A operand, so D = out^T
template <int MBW>
__device__ __forceinline__ void mfma_kstep(t_f4 (&C)[MBW][2], const uint4 (&a)[MBW][2], const t_h8 B00,
                                           const t_h8 B01, const t_h8 B10, const t_h8 B11, const t_h8 b00,
                                           const t_h8 b10) {
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    const t_h8 a0 = __builtin_bit_cast(t_h8, a[mb][0]);
    const t_h8 a1 = __builtin_bit_cast(t_h8, a[mb][1]);
    C[mb][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b00, a1, C[mb][0], 0, 0, 0);
    C[mb][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B01, a0, C[mb][0], 0, 0, 0);
    C[mb][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B00, a0, C[mb][0], 0, 0, 0);
    C[mb][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b10, a1, C[mb][1], 0, 0, 0);
    C[mb][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B11, a0, C[mb][1], 0, 0, 0);
    C[mb][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B10, a0, C[mb][1], 0, 0, 0);
  }
}

#ifndef AZ_T16_PF
#define AZ_T16_PF 2  // k-steps of B fragments in flight ahead of their MFMAs
#endif

// One conv phase's K loop: R residual k-steps (the block input's own rows x
// the 1x1 projection weights, k-steps 36.. of the conv2 pack, into accr),
// then 9 taps x 4 channel chunks of 32 (into acc).  The taps are a runtime
// loop with the chunks unrolled inside: fully unrolled, the two phases made
// a 110 KB kernel (the instruction cache holds 64 KB).  Ring slots are the
// k-step mod 4 (R is 0 or 4), so every register index stays static.
template <int MBW, int R>
__device__ __forceinline__ void k_loop(const uint4* __restrict__ act, const uint4* __restrict__ wmain,
                                       const uint4* __restrict__ wres, t_f4 (&acc)[MBW][2],
                                       t_f4 (&accr)[MBW][2], const int (&r_)[MBW], const int (&py_)[MBW],
                                       const int (&px_)[MBW], const bool (&valid_)[MBW], int H, int W,
                                       int zrow, int nq, int lane) {
  static_assert(R == 0 || R == 4, "ring slots = k-step mod 4");
  constexpr int PF = AZ_T16_PF, NB = 4;
  static_assert(PF >= 1 && PF <= 3, "prefetch depth");
  const int gq = lane >> 4;
  // the tap geometry laundered through an empty asm per call: the k-loops sit
  // in the runtime depth loop, and without this the compiler hoists every
  // k-step's LDS address out of it (loop invariant) and spills them
  int r[MBW], py[MBW], px[MBW];
  bool valid[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    r[mb] = r_[mb];
    py[mb] = py_[mb];
    px[mb] = px_[mb];
    int v = valid_[mb];
    asm volatile("" : "+v"(r[mb]), "+v"(py[mb]), "+v"(px[mb]), "+v"(v));
    valid[mb] = v != 0;
  }
  const uint4* wm = wmain + (size_t)(nq * 2) * 2 * 64 + lane;
  const uint4* wr = R ? wres + (size_t)(nq * 2) * 2 * 64 + lane + (size_t)36 * 1024 : nullptr;
  uint4 bq[NB][4];
  auto load_b = [&](const uint4* p, uint4(&dst)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q] = p[q * 64];
  };
  // k-step s of the phase -> its B fragments (s < R: residual)
  auto bsrc = [&](int s) { return s < R ? wr + (size_t)s * 1024 : wm + (size_t)(s - R) * 1024; };

  int abase[MBW], akey[MBW];
  auto set_own = [&]() {
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      abase[mb] = (valid[mb] ? r[mb] : zrow) * 32;
      akey[mb] = r[mb];
    }
  };
  auto set_tap = [&](int t) {  // runtime tap
    const int dy = t / 3 - 1, dx = t - (t / 3) * 3 - 1;
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      const bool ok = valid[mb] && py[mb] + dy >= 0 && py[mb] + dy < H && px[mb] + dx >= 0 && px[mb] + dx < W;
      const int sr = r[mb] + dy * W + dx;
      abase[mb] = (ok ? sr : zrow) * 32;
      akey[mb] = sr;  // also for the zero row: the lane keeps its bank quad
    }
  };
  uint4 aq[2][MBW][2];
  auto load_a = [&](int chunk, uint4(&dst)[MBW][2]) {
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      const int sl = phys_slot(akey[mb], 4 * chunk + gq);
      dst[mb][0] = act[abase[mb] + sl];
      dst[mb][1] = act[abase[mb] + 16 + sl];
    }
  };
  auto kstep = [&](t_f4(&C)[MBW][2], const uint4(&b)[4], const uint4(&a)[MBW][2]) {
    const t_h8 B00 = __builtin_bit_cast(t_h8, b[0]), B01 = __builtin_bit_cast(t_h8, b[1]);
    const t_h8 B10 = __builtin_bit_cast(t_h8, b[2]), B11 = __builtin_bit_cast(t_h8, b[3]);
    mfma_kstep<MBW>(C, a, B00, B01, B10, B11, unscale_b0(b[0]), unscale_b0(b[2]));
  };

#pragma unroll
  for (int k = 0; k < PF; ++k) load_b(bsrc(k), bq[k]);
  if (R) set_own();
  else set_tap(0);
  load_a(0, aq[0]);
  // ---- residual k-steps (static)
#pragma unroll
  for (int s = 0; s < R; ++s) {
    __builtin_amdgcn_sched_barrier(0);
    load_b(bsrc(s + PF), bq[(s + PF) % NB]);
    if (s + 1 < R) {
      load_a(s + 1, aq[(s + 1) & 1]);
    } else {
      set_tap(0);
      load_a(0, aq[(s + 1) & 1]);
    }
    kstep(accr, bq[s % NB], aq[s & 1]);
    __builtin_amdgcn_sched_group_barrier(0x0020, 4, 0);        // VMEM reads (B, PF ahead)
    __builtin_amdgcn_sched_group_barrier(0x0100, 2 * MBW, 0);  // DS reads (A, next k-step)
    __builtin_amdgcn_sched_group_barrier(0x0008, 6 * MBW, 0);  // MFMA
  }
  // ---- 9 taps x 4 chunks
#pragma unroll 1
  for (int t = 0; t < 9; ++t) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      __builtin_amdgcn_sched_barrier(0);
      // main k-step PF ahead (the prologue or the residual steps fetched 0 .. PF - 1)
      const int ahead = 4 * t + c + PF;
      if (c + PF < 4 || t < 8) load_b(wm + (size_t)ahead * 1024, bq[(c + PF) % NB]);
      if (c < 3) {
        load_a(c + 1, aq[(c + 1) & 1]);
      } else if (t < 8) {
        set_tap(t + 1);
        load_a(0, aq[0]);
      }
      kstep(acc, bq[c % NB], aq[c & 1]);
      __builtin_amdgcn_sched_group_barrier(0x0020, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x0100, 2 * MBW, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 6 * MBW, 0);
    }
  }
}

template <int MBW>
__global__ __launch_bounds__(kThreads, 2) void tower16_kernel(const TowerNet* __restrict__ net,
                                                               const Board* __restrict__ boards,
                                                               const float4* __restrict__ x,
                                                               const int* __restrict__ count, int n_static,
                                                               int H, int W, int A, int bpw,
                                                               float* __restrict__ probs,
                                                               float* __restrict__ values,
                                                               unsigned long long* __restrict__ err) {
  constexpr int TR = 32 * MBW;  // tile rows (two M halves of MBW 16-row blocks)
  extern __shared__ __attribute__((aligned(16))) uint4 act[];  // [TR + 1][32]: rows, then the zero row
  TowerSmem& sm = *reinterpret_cast<TowerSmem*>(act + (TR + 1) * 32);
  float* red = reinterpret_cast<float*>(&sm + 1);  // [TR][4][3] heads partial sums

  const int HW = H * W;
  const int n = count ? *count : n_static;
  const int b0 = blockIdx.x * bpw;
  if (b0 >= n) return;  // block-uniform
  const int nbrd = min(bpw, n - b0);
  const int live = nbrd * HW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int zrow = TR;
  const TowerNet& T = *net;

  if (tid < 32) act[zrow * 32 + tid] = make_uint4(0u, 0u, 0u, 0u);
  if (tid < 2) sm.flag[tid] = 0;
  __syncthreads();  // the flags before any layer may set one

  // ---------------------------------------------------------------- stem
  // conv3x3 4 -> F + folded BN + ReLU, fp32 on the VALU: the fmaf chain of
  // stem_conv_kernel (az_nn.hip), from the one-hot planes x or, bitwise the
  // same, from the boards (only the two nonzero terms per in-board tap)
  constexpr int NIS = TR * 32 / kThreads;
  int srow[NIS], scq[NIS], sbrd[NIS];
  float4 sy[NIS];
#pragma unroll
  for (int i = 0; i < NIS; ++i) {
    const int idx = tid + i * kThreads;
    const int rr = idx >> 5, cg = idx & 31;
    srow[i] = rr < live ? rr : -1;
    scq[i] = cg;
    sbrd[i] = 0;
    sy[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rr >= live) continue;
    const int b = rr / HW, p = rr - b * HW;
    sbrd[i] = b;
    const int y0 = p / W, x0 = p - y0 * W;
    float4 acc = reinterpret_cast<const float4*>(T.stem_b)[cg];
    const float4* ws = reinterpret_cast<const float4*>(T.stem_w);
    if (boards) {
      const Board bd = boards[b0 + b];
      const uint64_t own0 = bd.own[0], own1 = bd.own[1], opp0 = bd.opp[0], opp1 = bd.opp[1];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ny = y0 + tap / 3 - 1, nx = x0 + tap % 3 - 1;
        if (ny < 0 || ny >= H || nx < 0 || nx >= W) continue;
        const int q = ny * W + nx;
        const uint64_t ow = q < 64 ? own0 : own1, op = q < 64 ? opp0 : opp1;
        const int sh = q & 63;
        const int st = ((ow >> sh) & 1ull) ? 1 : (((op >> sh) & 1ull) ? 2 : 0);
        const float4 w1 = ws[(tap * 4 + st) * 32 + cg];
        const float4 w3 = ws[(tap * 4 + 3) * 32 + cg];
        acc.x = fmaf(1.0f, w1.x, acc.x);
        acc.y = fmaf(1.0f, w1.y, acc.y);
        acc.z = fmaf(1.0f, w1.z, acc.z);
        acc.w = fmaf(1.0f, w1.w, acc.w);
        acc.x = fmaf(1.0f, w3.x, acc.x);
        acc.y = fmaf(1.0f, w3.y, acc.y);
        acc.z = fmaf(1.0f, w3.z, acc.z);
        acc.w = fmaf(1.0f, w3.w, acc.w);
      }
    } else {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ny = y0 + tap / 3 - 1, nx = x0 + tap % 3 - 1;
        if (ny < 0 || ny >= H || nx < 0 || nx >= W) continue;
        const float4 v = x[(size_t)(b0 + b) * HW + ny * W + nx];
        const float vin[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 wv = ws[(tap * 4 + c) * 32 + cg];
          acc.x = fmaf(vin[c], wv.x, acc.x);
          acc.y = fmaf(vin[c], wv.y, acc.y);
          acc.z = fmaf(vin[c], wv.z, acc.z);
          acc.w = fmaf(vin[c], wv.w, acc.w);
        }
      }
    }
    sy[i] = make_float4(fmaxf(acc.x, 0.f), fmaxf(acc.y, 0.f), fmaxf(acc.z, 0.f), fmaxf(acc.w, 0.f));
  }
  int par = 0;
  // scale state: buffer contents X (block input) and H (conv1 output)
  bool anyX = store_layer<NIS>(act, srow, scq, sbrd, sy, sm, par, sm.sc[0], nbrd, err);
  bool anyH = false;
  par ^= 1;

  // ---------------------------------------------------------------- tower
  const int mh = wave >> 2, nq = wave & 3, r16 = lane & 15, gq = lane >> 4;
  int r[MBW], py[MBW], px[MBW], brd[MBW];
  bool valid[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    r[mb] = (mh * MBW + mb) * 16 + r16;
    valid[mb] = r[mb] < live;
    const int b = valid[mb] ? r[mb] / HW : 0;
    brd[mb] = b;
    const int p = r[mb] - b * HW;
    py[mb] = p / W;
    px[mb] = p - py[mb] * W;
  }
  int orow[2 * MBW], ocq[2 * MBW], obrd[2 * MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      orow[mb * 2 + nb] = valid[mb] ? r[mb] : -1;
      ocq[mb * 2 + nb] = 8 * nq + 4 * nb + gq;
      obrd[mb * 2 + nb] = brd[mb];
    }
  const int depth = T.depth;
  t_f4 acc[MBW][2], accr[MBW][2];
  float4 yv[2 * MBW];
  for (int d = 0; d < depth; ++d) {
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        acc[mb][nb] = t_f4{0.f, 0.f, 0.f, 0.f};
        accr[mb][nb] = t_f4{0.f, 0.f, 0.f, 0.f};
      }
    // conv1 (+ the projection residual into accr), input X
    k_loop<MBW, 4>(act, T.k1[d], T.k2[d], acc, accr, r, py, px, valid, H, W, zrow, nq, lane);
    __syncthreads();  // every wave is done reading X: H overwrites it
    {
      const float osc = T.s1[d];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const float4 bc = *reinterpret_cast<const float4*>(T.b1[d] + 32 * nq + 16 * nb + 4 * gq);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          const float o = anyX ? ldexpf(osc, sm.sc[0][brd[mb]]) : osc;
          const t_f4 a = acc[mb][nb];
          yv[mb * 2 + nb] = make_float4(fmaxf(fmaf(a[0], o, bc.x), 0.f), fmaxf(fmaf(a[1], o, bc.y), 0.f),
                                        fmaxf(fmaf(a[2], o, bc.z), 0.f), fmaxf(fmaf(a[3], o, bc.w), 0.f));
        }
      }
    }
    anyH = store_layer<2 * MBW>(act, orow, ocq, obrd, yv, sm, par, sm.sc[1], nbrd, err);
    par ^= 1;
    // the residual was accumulated at X's scale, conv2 runs at H's
    if (anyX || anyH) {
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        const int e = (anyX ? sm.sc[0][brd[mb]] : 0) - (anyH ? sm.sc[1][brd[mb]] : 0);
        if (e) {
          const float f = ldexpf(1.f, e);
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) accr[mb][nb] *= f;
        }
      }
    }
    // conv2 on H, on top of the residual
    k_loop<MBW, 0>(act, T.k2[d], nullptr, accr, accr, r, py, px, valid, H, W, zrow, nq, lane);
    const float osc = T.s2[d];
    if (d + 1 < depth) {
      __syncthreads();  // every wave is done reading H: the block output overwrites it
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const float4 bc = *reinterpret_cast<const float4*>(T.b2[d] + 32 * nq + 16 * nb + 4 * gq);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          const float o = anyH ? ldexpf(osc, sm.sc[1][brd[mb]]) : osc;
          const t_f4 a = accr[mb][nb];
          yv[mb * 2 + nb] = make_float4(fmaxf(fmaf(a[0], o, bc.x), 0.f), fmaxf(fmaf(a[1], o, bc.y), 0.f),
                                        fmaxf(fmaf(a[2], o, bc.z), 0.f), fmaxf(fmaf(a[3], o, bc.w), 0.f));
        }
      }
      anyX = store_layer<2 * MBW>(act, orow, ocq, obrd, yv, sm, par, sm.sc[0], nbrd, err);
      par ^= 1;
      continue;
    }
    // ------------------------------------------------------------ heads
    // last block: its output goes straight into the 1x1 head convs (policy
    // F -> 2, value F -> 1, folded BN, ReLU; model.py:68-149): per lane its 8
    // channels, a fixed xor tree over the four lane groups, the four N
    // quarters in order through LDS
    float s3[MBW][3];
    {
      float hw[2][4][3];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int c = 32 * nq + 16 * nb + 4 * gq + v;
          hw[nb][v][0] = T.wpc[2 * c];
          hw[nb][v][1] = T.wpc[2 * c + 1];
          hw[nb][v][2] = T.wvc[c];
        }
      float4 bc[2];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) bc[nb] = *reinterpret_cast<const float4*>(T.b2[d] + 32 * nq + 16 * nb + 4 * gq);
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        const float o = anyH ? ldexpf(osc, sm.sc[1][brd[mb]]) : osc;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const float yy = fmaxf(fmaf(accr[mb][nb][v], o, (&bc[nb].x)[v]), 0.f);
            a0 = fmaf(yy, hw[nb][v][0], a0);
            a1 = fmaf(yy, hw[nb][v][1], a1);
            a2 = fmaf(yy, hw[nb][v][2], a2);
          }
        a0 += __shfl_xor(a0, 16);
        a1 += __shfl_xor(a1, 16);
        a2 += __shfl_xor(a2, 16);
        a0 += __shfl_xor(a0, 32);
        a1 += __shfl_xor(a1, 32);
        a2 += __shfl_xor(a2, 32);
        s3[mb][0] = a0;
        s3[mb][1] = a1;
        s3[mb][2] = a2;
      }
    }
    if (gq == 0)
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb)
        if (valid[mb])
#pragma unroll
          for (int k = 0; k < 3; ++k) red[(r[mb] * 4 + nq) * 3 + k] = s3[mb][k];
  }
  __syncthreads();  // red complete; the activation rows are no longer read

  // flattened head features per board (Keras Flatten of NHWC: [p][c]) in the
  // activation area: pf [bpw][2HW], vf [bpw][HW], logits [bpw][A]
  float* pf = reinterpret_cast<float*>(act);
  float* vf = pf + bpw * 2 * HW;
  float* lg = vf + bpw * HW;
  const float bpc0 = T.bpc[0], bpc1 = T.bpc[1], bvc0 = T.bvc[0];
  for (int rr = tid; rr < live; rr += kThreads) {
    const int b = rr / HW, p = rr - b * HW;
    float t[3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
      t[k] = ((red[(rr * 4 + 0) * 3 + k] + red[(rr * 4 + 1) * 3 + k]) + red[(rr * 4 + 2) * 3 + k]) +
             red[(rr * 4 + 3) * 3 + k];
    pf[b * 2 * HW + 2 * p] = fmaxf(t[0] + bpc0, 0.f);
    pf[b * 2 * HW + 2 * p + 1] = fmaxf(t[1] + bpc1, 0.f);
    vf[b * HW + p] = fmaxf(t[2] + bvc0, 0.f);
  }
  __syncthreads();
  // policy Dense(A) logits, one thread per (board, action)
  for (int idx = tid; idx < nbrd * A; idx += kThreads) {
    const int b = idx / A, a = idx - b * A;
    float s = T.bpd[a];
    const float* pb = pf + b * 2 * HW;
    for (int i = 0; i < 2 * HW; ++i) s = fmaf(pb[i], T.wpd[i * A + a], s);
    lg[b * A + a] = s;
  }
  // value Dense(hidden) ReLU -> Dense(1): thread j of each 256-thread half,
  // boards half, half + 2, ...; its weight column read once for all of them
  {
    const int j = tid & 255, half = tid >> 8;
    const int hidden = T.hidden;
    float sv[kTowerMaxBoards / 2];
#pragma unroll
    for (int k = 0; k < kTowerMaxBoards / 2; ++k) sv[k] = j < hidden ? T.bv1[j] : 0.f;
    if (j < hidden)
      for (int p = 0; p < HW; ++p) {
        const float w = T.wv1[p * hidden + j];
#pragma unroll
        for (int k = 0; k < kTowerMaxBoards / 2; ++k) {
          const int b = half + 2 * k;
          if (b < nbrd) sv[k] = fmaf(vf[b * HW + p], w, sv[k]);
        }
      }
    const float w2 = j < hidden ? T.wv2[j] : 0.f;
#pragma unroll
    for (int k = 0; k < kTowerMaxBoards / 2; ++k) {
      const int b = half + 2 * k;
      if (b >= nbrd) break;  // wave-uniform
      const float part = wsum(fmaxf(sv[k], 0.f) * w2);
      if (lane == 0) sm.vred[b][wave & 3] = part;
    }
  }
  __syncthreads();
  // softmax (one wave per board) and tanh
  if (wave < nbrd) {
    const int b = wave;
    float m = -INFINITY;
    for (int a = lane; a < A; a += 64) m = fmaxf(m, lg[b * A + a]);
    m = wmax(m);
    float z = 0.f;
    for (int a = lane; a < A; a += 64) z += expf(lg[b * A + a] - m);
    z = wsum(z);
    for (int a = lane; a < A; a += 64) probs[(size_t)(b0 + b) * A + a] = expf(lg[b * A + a] - m) / z;
    if (lane == 0)
      values[b0 + b] = tanhf((((sm.vred[b][0] + sm.vred[b][1]) + sm.vred[b][2]) + sm.vred[b][3]) + T.bv2[0]);
  }
}

}  // namespace

int tower16_tile_rows(int HW) {
  // 128-row tiles unless 96 rows hold the same boards (more rows per tile, same work per board)
  if (HW > 128) return 0;
  const int b128 = std::min(128 / HW, kTowerMaxBoards), b96 = std::min(96 / HW, kTowerMaxBoards);
  if (b96 >= 1 && b96 * HW * 128 >= b128 * HW * 96) return 96;  // 96-row tiles are at least as full
  return 128;
}

int tower16_boards_per_tile(int HW) {
  const int tr = tower16_tile_rows(HW);
  return tr ? std::min(tr / HW, kTowerMaxBoards) : 0;
}

size_t tower16_lds_bytes(int HW) {
  const int tr = tower16_tile_rows(HW);
  return (size_t)(tr + 1) * 512 + sizeof(TowerSmem) + (size_t)tr * 4 * 3 * sizeof(float);
}

template <int MBW>
static void launch_mbw(const TowerNet* net, const Board* boards, const float4* x, const int* count, int n_max,
                       int H, int W, int A, float* probs, float* values, unsigned long long* err,
                       hipStream_t s) {
  const int bpw = tower16_boards_per_tile(H * W);
  const int grid = (n_max + bpw - 1) / bpw;
  const size_t bytes = tower16_lds_bytes(H * W);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tower16_kernel<MBW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    attr = true;
  }
  tower16_kernel<MBW><<<grid, kThreads, bytes, s>>>(net, boards, x, count, n_max, H, W, A, bpw, probs, values,
                                                     err);
}

void launch_tower16(const TowerNet* net, const Board* boards, const float4* x, const int* count, int n_max,
                    int H, int W, int A, float* probs, float* values, unsigned long long* err, hipStream_t s) {
  if (n_max <= 0) return;
  if (tower16_tile_rows(H * W) == 96)
    launch_mbw<3>(net, boards, x, count, n_max, H, W, A, probs, values, err, s);
  else
    launch_mbw<4>(net, boards, x, count, n_max, H, W, A, probs, values, err, s);
}

}  // namespace az
