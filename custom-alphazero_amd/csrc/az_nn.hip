// az_nn.hip -- batched policy/value forward for gfx950.
//
// Network = the reference's Keras PolicyValueModel at inference
// (custom_alphazero/model/tensorflow/model.py:152-188, base_layers.py:20-125):
//   stem   conv3x3 4->F + BN + ReLU                       (InnerConvBlock)
//   depth x OuterConvBlock: conv3x3+BN+ReLU, conv3x3+BN, + conv1x1+BN of the
//          block input (projection residual), ReLU
//   policy conv1x1 F->2 + BN + ReLU, flatten HWC, Dense(A) softmax
//   value  conv1x1 F->1 + BN + ReLU, flatten, Dense(256) ReLU, Dense(1) tanh
// BatchNorm runs with moving statistics (call(training=False)); the engine
// folds it into the conv weights on the host (az_engine.hip).
//
// Kernels (each one's roofline in DESIGN.md):
//   encode_boards    Board.full_state for the eval queue (HBM/latency bound)
//   stem_conv        K = 36, VALU; writes split16 rows (AZ_CONV_F16X2) or fp32
//   conv16_kernel    the tower's 3x3 convs, default (az_conv16.hip)
//   conv3x3_mfma     AZ_CONV_DIRECT: implicit GEMM on v_mfma_f32_32x32x2_f32
//                    (exact f32 FMA chains): M = boards*HW rows, N = F, K = 9F
//                    (+F for the fused 1x1 projection residual).  MFMA bound.
//   heads            one wave per board
// Reduction order is fixed per output element and independent of the batch,
// so a board's outputs do not depend on what else is in the batch.
#include <stdlib.h>

#include <algorithm>

#include "az_nn.h"
#include "az_tree.h"

namespace az {

// ------------------------------------------------------------------ encode
// x[b][p][4] = [empty, own, opp, 1] (connect_n/board.py:83-98: np.eye(3)
// indexed by the canonical array -> channels 0:empty, 1:+1, 2:-1; plane 3 is
// `turn`, always +1 under keep_same_player).
__global__ void encode_boards_kernel(const Board* __restrict__ boards, const int* __restrict__ count,
                                     int n_static, int HW, float4* __restrict__ x) {
  const int n = count ? *count : n_static;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * HW) return;
  const int b = idx / HW, p = idx - b * HW;
  const Board bd = boards[b];
  const float own = bit(bd.own, p) ? 1.0f : 0.0f;
  const float opp = bit(bd.opp, p) ? 1.0f : 0.0f;
  x[idx] = make_float4(1.0f - own - opp, own, opp, 1.0f);
}

// legal-move mask in action order (board.py:154-155)
__global__ void legal_mask_kernel(const Board* __restrict__ boards, int n, GameCfg g,
                                  uint8_t* __restrict__ mask) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * g.A) return;
  const int b = idx / g.A, a = idx - b * g.A;
  mask[idx] = action_cell(g, boards[b], a) >= 0;
}

// -------------------------------------------------------------------- stem
// conv3x3 4 -> F with 'same' zero padding, folded BN, ReLU.  One thread per
// (row, 4 output channels).  ws: [36][F] with k = tap*4 + c, tap = ky*3+kx.
template <int F, bool SPLIT>
__global__ __launch_bounds__(256) void stem_conv_kernel(const float4* __restrict__ x,
                                                        const float* __restrict__ ws,
                                                        const float* __restrict__ bias,
                                                        const int* __restrict__ count, int n_static,
                                                        int H, int W, void* __restrict__ out,
                                                        unsigned long long* __restrict__ err) {
  // weights (18 KB) are read through L1 by every thread: no per-block LDS
  // staging (which cost ~18 KB of L2 traffic per 256 outputs)
  constexpr int G4 = F / 4;
  const int n = count ? *count : n_static;
  const int HW = H * W;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * HW * G4) return;
  const int r = idx / G4, cg = idx - r * G4;
  const int b = r / HW, p = r - b * HW;
  const int y = p / W, xx = p - y * W;
  float4 acc = *reinterpret_cast<const float4*>(bias + cg * 4);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int ny = y + tap / 3 - 1, nx = xx + tap % 3 - 1;
    if (ny < 0 || ny >= H || nx < 0 || nx >= W) continue;
    const float4 v = x[b * HW + ny * W + nx];
    const float vin[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 wv = *reinterpret_cast<const float4*>(ws + (tap * 4 + c) * F + cg * 4);
      acc.x += vin[c] * wv.x;
      acc.y += vin[c] * wv.y;
      acc.z += vin[c] * wv.z;
      acc.w += vin[c] * wv.w;
    }
  }
  acc.x = fmaxf(acc.x, 0.0f);
  acc.y = fmaxf(acc.y, 0.0f);
  acc.z = fmaxf(acc.z, 0.0f);
  acc.w = fmaxf(acc.w, 0.0f);
  if (SPLIT && err && !(fmaxf(fmaxf(acc.x, acc.y), fmaxf(acc.z, acc.w)) <= 32752.f)) atomicOr(err, kErrActRange);
  store_act4<SPLIT>(out, (size_t)r, cg, acc);
}

// Same layer straight from the boards (self-play): the input is one-hot, so
// each in-board tap contributes w[tap][state] then w[tap][3] (the turn
// plane) -- exactly the nonzero terms of stem_conv_kernel's fmaf chain in its
// channel order (a zero term leaves the accumulator unchanged: it is never
// -0), so outputs are bitwise those of encode + stem_conv.  Saves the encode
// pass and the float4 input reads.
// Blocks loop over pixels (8 per pass: lane group = 32 channel quads) with
// the 18 KB of stem weights staged once per block in LDS (read per pixel
// through L1 the kernel was L1-bandwidth bound).
// Copy n floats from global memory into LDS with the whole workgroup (256
// threads), 8 loads per thread in flight per batch (float4 when both sides
// are 16-byte aligned).  A rolled one-float-per-iteration loop waits for each
// load before its LDS store: the Connect-4 heads kernel staged its 45 KB of
// dense weights in 45 serialized L2 round trips.
__device__ __forceinline__ void stage_lds(float* dst, const float* __restrict__ src, int n) {
  const int t = threadIdx.x;
  if ((n & 3) == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    const int n4 = n >> 2;
    for (int base = 0; base < n4; base += 8 * 256) {
      float4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = s4[min(base + t + k * 256, n4 - 1)];  // clamped: no guard
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int j = base + t + k * 256;
        if (j < n4) d4[j] = v[k];
      }
    }
  } else {
    for (int base = 0; base < n; base += 8 * 256) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = src[min(base + t + k * 256, n - 1)];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int j = base + t + k * 256;
        if (j < n) dst[j] = v[k];
      }
    }
  }
}

template <int F, bool SPLIT>
__global__ __launch_bounds__(256) void stem_board_kernel(const Board* __restrict__ boards,
                                                         const float* __restrict__ ws,
                                                         const float* __restrict__ bias,
                                                         const int* __restrict__ count, int n_static,
                                                         int H, int W, void* __restrict__ out,
                                                         unsigned long long* __restrict__ err) {
  constexpr int G4 = F / 4;
  static_assert(256 % G4 == 0, "a pass covers whole pixels");
  constexpr int PPB = 256 / G4;  // pixels per pass
  __shared__ float4 wsh[36 * G4];
  const int n = count ? *count : n_static;
  const int HW = H * W;
  const int npix = n * HW;
  if ((int)blockIdx.x * PPB >= npix) return;  // block-uniform
  stage_lds(reinterpret_cast<float*>(wsh), ws, 36 * G4 * 4);
  __syncthreads();
  const int cg = threadIdx.x % G4;
  const float4 b4 = reinterpret_cast<const float4*>(bias)[cg];
  for (int r = blockIdx.x * PPB + threadIdx.x / G4; r < npix; r += gridDim.x * PPB) {
    const int b = r / HW, p = r - b * HW;
    const int y = p / W, xx = p - y * W;
    // the board's words as scalars: indexing own[q >> 6] put the Board in
    // scratch (40 B per lane, 51 us per launch at 1940 boards)
    const Board bd = boards[b];
    const uint64_t own0 = bd.own[0], own1 = bd.own[1], opp0 = bd.opp[0], opp1 = bd.opp[1];
    float4 acc = b4;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ny = y + tap / 3 - 1, nx = xx + tap % 3 - 1;
      if (ny < 0 || ny >= H || nx < 0 || nx >= W) continue;
      const int q = ny * W + nx;
      const uint64_t ow = q < 64 ? own0 : own1, op = q < 64 ? opp0 : opp1;
      const int sh = q & 63;
      const int st = ((ow >> sh) & 1ull) ? 1 : (((op >> sh) & 1ull) ? 2 : 0);
      const float4 w1 = wsh[(tap * 4 + st) * G4 + cg];
      const float4 w3 = wsh[(tap * 4 + 3) * G4 + cg];
      acc.x = fmaf(1.0f, w1.x, acc.x);
      acc.y = fmaf(1.0f, w1.y, acc.y);
      acc.z = fmaf(1.0f, w1.z, acc.z);
      acc.w = fmaf(1.0f, w1.w, acc.w);
      acc.x = fmaf(1.0f, w3.x, acc.x);
      acc.y = fmaf(1.0f, w3.y, acc.y);
      acc.z = fmaf(1.0f, w3.z, acc.z);
      acc.w = fmaf(1.0f, w3.w, acc.w);
    }
    acc.x = fmaxf(acc.x, 0.0f);
    acc.y = fmaxf(acc.y, 0.0f);
    acc.z = fmaxf(acc.z, 0.0f);
    acc.w = fmaxf(acc.w, 0.0f);
    // the split16 row format holds |x| <= 32752 (the per-layer convs flag theirs too)
    if (SPLIT && err && !(fmaxf(fmaxf(acc.x, acc.y), fmaxf(acc.z, acc.w)) <= 32752.f)) atomicOr(err, kErrActRange);
    store_act4<SPLIT>(out, (size_t)r, cg, acc);
  }
}

// ------------------------------------------------------------ conv3x3 MFMA
// out[r][n] = ReLU( sum_k A[r][k] * W[k][n] + bias[n] )
//   k in [0, 9F): A = in[neighbour(r, tap)][c], tap = k / F, c = k % F
//   k in [9F, 10F) (RESIDUAL): A = res_in[r][c]  (fused 1x1 projection)
//
// Workgroup = 4 waves = a 32-row x 128-column output tile; wave w owns
// columns [32w, +32).
//   * A: the tile's input rows plus a halo of W+1 rows on each side are staged
//     ONCE into LDS (the "slab"); every tap reads its shifted view of it, and
//     off-board neighbours read a zero row (the fused residual's block-input
//     rows are staged beside it).  Rows are 128 floats = 32 16-byte
//     chunks, chunk j of slab row r stored at j ^ (r & 15): the 16 distinct
//     rows a ds_read_b128 lane group touches land on 16 distinct bank quads.
//   * B: weights are pre-packed on the host in MFMA fragment order
//     ([chunk][tile][q][lane] float4, az_engine.hip pack_fragments) and stream
//     straight into registers with fully coalesced 1 KiB loads, one 32-wide K
//     chunk ahead -- no LDS, no barrier in the K loop.
// v_mfma_f32_32x32x2_f32 is an exact f32 FMA chain; inside a chunk lane half
// h owns k = 16h..16h+15 and k-step s sums the pair (s, 16+s): a fixed order
// per output element, independent of the batch.
constexpr int kChunkK = 32;

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int slab_swz(int chunk, int key) {
  return (chunk & 16) | ((chunk ^ key) & 15);
}

size_t conv_lds_bytes(int TR, int W, bool residual) {
  const int slab_rows = TR + 2 * (W + 1);
  return (size_t)(slab_rows + 1 + (residual ? TR : 0)) * 512;
}

// One 32x32 MFMA tile per wave: the four waves take 32-column slices of a
// 32-row x 128-column output tile.  (Round-1 A/B, DESIGN.md: wider tiles,
// A read one chunk ahead, the residual rows from global and 3-4 waves/SIMD
// all measured slower and were removed.)
template <int F, bool RESIDUAL>
__global__ __launch_bounds__(256, 2) void conv3x3_mfma_kernel(
    const float* __restrict__ in, const float* __restrict__ res_in,
    const float4* __restrict__ wpack, const float* __restrict__ bias, float* __restrict__ out,
    const int* __restrict__ count, int n_static, int H, int W) {
  static_assert(F == 128, "tile assumes F = 128 channels (32 16-byte chunks per row)");
  constexpr int NCH = (RESIDUAL ? 10 : 9) * (F / kChunkK);
  constexpr int TR = 32;
  extern __shared__ __attribute__((aligned(16))) float4 lds4[];

  const int HW = H * W, halo = W + 1;
  const int n_boards = count ? *count : n_static;
  const int rows = n_boards * HW;
  const int row0 = blockIdx.x * TR;
  if (row0 >= rows) return;
  const int tid = threadIdx.x;
  const int slab_rows = TR + 2 * halo;
  float4* slab = lds4;
  float4* zero_row = lds4 + slab_rows * 32;
  float4* xslab = zero_row + 32;

  // ---- stage the slab (and the residual rows) once
  const float4* in4 = reinterpret_cast<const float4*>(in);
  for (int i = tid; i < slab_rows * 32; i += 256) {
    const int r = i >> 5, j = i & 31, g = row0 - halo + r;
    const float4 v = (g >= 0 && g < rows) ? in4[(size_t)g * 32 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
    slab[r * 32 + slab_swz(j, r)] = v;
  }
  if (tid < 32) zero_row[tid] = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (RESIDUAL) {
    const float4* x4 = reinterpret_cast<const float4*>(res_in);
    for (int i = tid; i < TR * 32; i += 256) {
      const int r = i >> 5, j = i & 31, g = row0 + r;
      const float4 v = g < rows ? x4[(size_t)g * 32 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
      xslab[r * 32 + slab_swz(j, r)] = v;
    }
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int rl = r32;  // local row of this lane's A operand
  const int grow = row0 + rl;
  const int pos = grow % HW;
  const int py = pos / W, px = pos - (pos / W) * W;
  const bool row_ok = grow < rows;

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;

  // B fragment stream: float4 index ((c*4 + tile)*4 + q)*64 + lane.  Two
  // register buffers in ping-pong (the loop is unrolled by two, so no copy):
  // chunk c+1's loads are first consumed a whole chunk of MFMAs later.
  const float4* wl = wpack + (size_t)wave * 256 + lane;
  float4 b0[4], b1[4];
  auto load_b = [&](int c, float4 (&dst)[4]) {
    const float4* wn = wl + (size_t)c * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q] = wn[q * 64];
  };
  auto load_a = [&](int c, float4 (&dst)[4]) {
    const int tap = c >> 2;
    const float4* base;
    int key;
    if (!RESIDUAL || tap < 9) {
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const bool ok = row_ok && py + dy >= 0 && py + dy < H && px + dx >= 0 && px + dx < W;
      const int sr = rl + halo + dy * W + dx;
      base = ok ? slab + sr * 32 : zero_row;
      key = ok ? (sr & 15) : 0;
    } else {
      base = xslab + rl * 32;
      key = rl & 15;
    }
    const int cbase = (c & 3) * 8 + h * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q] = base[slab_swz(cbase + q, key)];
  };
  auto compute = [&](const float4 (&a4)[4], const float4 (&bc)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[q].x, bc[q].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[q].y, bc[q].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[q].z, bc[q].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[q].w, bc[q].w, acc, 0, 0, 0);
    }
  };
  static_assert(NCH % 2 == 0, "ping-pong loop needs an even chunk count");
  float4 a0[4], a1[4];
  load_b(0, b0);
  // fully unrolled: no loop back-edge, so the waitcnt pass sees exactly which
  // loads each MFMA needs; tap geometry folds to constants per chunk
#pragma unroll
  for (int c = 0; c < NCH; c += 2) {
    load_b(c + 1, b1);
    load_a(c, a0);
    compute(a0, b0);
    if (c + 2 < NCH) load_b(c + 2, b0);
    load_a(c + 1, a1);
    compute(a1, b1);
  }

  // epilogue: C/D map col = lane&31, row = (i&3) + 8*(i>>2) + 4*h
  const int col = wave * 32 + r32;
  const float bcol = bias[col];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = row0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (row < rows) out[(size_t)row * F + col] = fmaxf(acc[i] + bcol, 0.0f);
  }
}

// ------------------------------------------------------------------- heads
// One wave per board.  Policy: conv1x1 F->2 (+BN folded) ReLU, flatten in
// (H, W, C) order (Keras Flatten on NHWC), Dense(A), softmax.  Value: conv1x1
// F->1 ReLU, Dense(hidden) ReLU, Dense(1) tanh (model.py:68-149).
struct HeadWeights {
  const float* wpc;  // [F][2]
  const float* bpc;  // [2]
  const float* wvc;  // [F]
  const float* bvc;  // [1]
  const float* wpd;  // [2*HW][A]
  const float* bpd;  // [A]
  const float* wv1;  // [HW][hidden]
  const float* bv1;  // [hidden]
  const float* wv2;  // [hidden]
  const float* bv2;  // [1]
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// FEAT: the 1x1 head convs already ran in the last conv's epilogue (feat =
// [boards][HW] float4 from conv16_kernel<.., HEADS>); same fmaf chains.
// Blocks loop over boards (4 per pass, one per wave); with STAGE the dense
// layers' weights (policy [2HW][A], value1 [HW][hidden]) are copied into LDS
// once per block instead of being re-read through L1 for every board.  The
// per-board arithmetic is unchanged.
template <int F, bool FEAT, bool STAGE, int AMAX>
__global__ __launch_bounds__(256) void heads_kernel(const float* __restrict__ act, HeadWeights hw,
                                                    const int* __restrict__ count, int n_static,
                                                    int HW, int A, int hidden,
                                                    float* __restrict__ probs,
                                                    float* __restrict__ values) {
  __shared__ float pflat[4][2 * kMaxCells];
  __shared__ float vflat[4][kMaxCells];
  __shared__ float logits[4][AMAX];  // AMAX = kMaxActions, or 2048 for chess (A = 1880)
  extern __shared__ float wsm[];
  const int n = count ? *count : n_static;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float* wpd = hw.wpd;
  const float* wv1 = hw.wv1;
  if constexpr (STAGE) {
    if ((int)blockIdx.x * 4 >= n) return;  // block-uniform
    const int npd = 2 * HW * A, nv1 = HW * hidden;
    stage_lds(wsm, hw.wpd, npd);
    stage_lds(wsm + npd, hw.wv1, nv1);
    __syncthreads();
    wpd = wsm;
    wv1 = wsm + npd;
  }
  for (int b = blockIdx.x * 4 + wave; b < n; b += gridDim.x * 4) {  // wave-uniform
  if constexpr (FEAT) {
    const float4* feat = reinterpret_cast<const float4*>(act) + (size_t)b * HW;
    for (int p = lane; p < HW; p += 64) {
      const float4 f = feat[p];
      pflat[wave][2 * p] = f.x;
      pflat[wave][2 * p + 1] = f.y;
      vflat[wave][p] = f.z;
    }
  }
  const float* base = act + (size_t)b * HW * F;
  for (int p = lane; p < HW && !FEAT; p += 64) {
    const float4* row = reinterpret_cast<const float4*>(base + (size_t)p * F);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll 8
    for (int q = 0; q < F / 4; ++q) {
      const float4 v = row[q];
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * q + e;
        s0 = fmaf(vv[e], hw.wpc[2 * c], s0);
        s1 = fmaf(vv[e], hw.wpc[2 * c + 1], s1);
        s2 = fmaf(vv[e], hw.wvc[c], s2);
      }
    }
    pflat[wave][2 * p] = fmaxf(s0 + hw.bpc[0], 0.f);
    pflat[wave][2 * p + 1] = fmaxf(s1 + hw.bpc[1], 0.f);
    vflat[wave][p] = fmaxf(s2 + hw.bvc[0], 0.f);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // policy dense + softmax
  for (int a = lane; a < A; a += 64) {
    float s = hw.bpd[a];
    for (int i = 0; i < 2 * HW; ++i) s += pflat[wave][i] * wpd[i * A + a];
    logits[wave][a] = s;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  float m = -INFINITY;
  for (int a = lane; a < A; a += 64) m = fmaxf(m, logits[wave][a]);
  m = wave_max(m);
  float z = 0.f;
  for (int a = lane; a < A; a += 64) z += expf(logits[wave][a] - m);
  z = wave_sum(z);
  for (int a = lane; a < A; a += 64) probs[(size_t)b * A + a] = expf(logits[wave][a] - m) / z;
  // value dense(hidden) ReLU -> dense(1) tanh
  float part = 0.f;
  for (int j = lane; j < hidden; j += 64) {
    float s = hw.bv1[j];
    for (int p = 0; p < HW; ++p) s += vflat[wave][p] * wv1[p * hidden + j];
    part += fmaxf(s, 0.f) * hw.wv2[j];
  }
  part = wave_sum(part);
  if (lane == 0) values[b] = tanhf(part + hw.bv2[0]);
  __builtin_amdgcn_wave_barrier();  // pflat/vflat/logits are reused by the next board
  }
}

// Chess-size heads (A = 1880), used when the 1x1 head convs ran in the last
// conv's epilogue (feat = [boards][HW] float4: policy ch 0, ch 1, value, 0).
// policy_dense_kernel: Dense(2HW -> A) as a tiled GEMM over the live batch --
// a workgroup owns 64 actions x 4NB boards, stages the weight tile [2HW][64]
// and the boards' flattened policy features [4NB][2HW] in LDS, and each thread
// accumulates one action for NB boards, s = bias + sum_i p[i] * w[i][a] in i
// order, into `logits` (the probs buffer).  One wave per board could not hide
// the 962 KB weight stream (60% of a chess step); here every weight is read
// once per 4NB boards.  NB = 8 (32 boards) for large launches; a self-play
// lane's 128 boards take NB = 2: 4x the workgroups (480), a quarter of the
// FMA chain per thread -- the launch is latency-bound, on the lane's chain.
template <int K, int NB>
__device__ __forceinline__ void policy_dense_body(const float4* __restrict__ feat, const float* __restrict__ wpd,
                                                  const float* __restrict__ bpd, const int* __restrict__ count,
                                                  int n_static, int HW, int A, float* __restrict__ logits) {
  __shared__ __attribute__((aligned(16))) float ws[K][64];
  __shared__ __attribute__((aligned(16))) float ps[4 * NB][K];
  const int n = count ? *count : n_static;
  const int a0 = blockIdx.x * 64, b0 = blockIdx.y * 4 * NB;
  if (b0 >= n) return;  // block-uniform
  const int t = threadIdx.x;
  // the tile's weight slab is contiguous (NetDev::pd_wt): 8 float4 loads per
  // thread, all in flight together (scalar loads from the [K][A] matrix, each
  // awaited before its LDS store, took 13 of the kernel's 17.7 us)
  {
    const float4* src = reinterpret_cast<const float4*>(wpd) + (size_t)blockIdx.x * K * 16;
    float4 v[K * 16 / 256];
#pragma unroll
    for (int k = 0; k < K * 16 / 256; ++k) v[k] = src[t + 256 * k];
#pragma unroll
    for (int k = 0; k < K * 16 / 256; ++k) {
      const int idx = t + 256 * k;
      *reinterpret_cast<float4*>(&ws[idx >> 4][(idx & 15) * 4]) = v[k];
    }
  }
  constexpr int HWK = K / 2;  // the launcher passes K = 2 * HW
#pragma unroll
  for (int k = 0; k < 4 * NB * HWK / 256; ++k) {
    const int idx = t + 256 * k;
    const int b = idx / HWK, p = idx - b * HWK;
    const float4 f = feat[(size_t)min(b0 + b, n - 1) * HWK + p];  // clamped (rows past n unused)
    ps[b][2 * p] = f.x;
    ps[b][2 * p + 1] = f.y;
  }
  __syncthreads();
  const int a = t & 63, bg = (t >> 6) * NB;
  if (a0 + a >= A) return;
  const float bias = bpd[a0 + a];
  float acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = bias;
  // the 8 boards' features as float4 over i (wave-uniform rows: LDS
  // broadcasts), 12 LDS reads per 32 FMAs instead of 36; same FMA order
  for (int i = 0; i < 2 * HW; i += 4) {
    const float w0 = ws[i][a], w1 = ws[i + 1][a], w2 = ws[i + 2][a], w3 = ws[i + 3][a];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const float4 f = *reinterpret_cast<const float4*>(&ps[bg + j][i]);
      acc[j] = fmaf(f.x, w0, acc[j]);
      acc[j] = fmaf(f.y, w1, acc[j]);
      acc[j] = fmaf(f.z, w2, acc[j]);
      acc[j] = fmaf(f.w, w3, acc[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (b0 + bg + j < n) logits[(size_t)(b0 + bg + j) * A + a0 + a] = acc[j];
}

template <int K, int NB>
__global__ __launch_bounds__(256) void policy_dense_kernel(const float4* __restrict__ feat,
                                                           const float* __restrict__ wpd,
                                                           const float* __restrict__ bpd,
                                                           const int* __restrict__ count, int n_static,
                                                           int HW, int A, float* __restrict__ logits) {
  policy_dense_body<K, NB>(feat, wpd, bpd, count, n_static, HW, A, logits);
}

// softmax over the logits in place + the value head (Dense(hidden) ReLU ->
// Dense(1) tanh), one board per 256-thread workgroup: a thread holds 8 of
// the board's logits in registers (one read, one exp, one write per logit)
// and owns hidden unit j of the value layer, whose weights it reads straight
// from L2 (each p a coalesced 1 KB row across the workgroup).  Block
// reductions: wave shuffles, then the 4 waves' partials through LDS.
// (4 boards per workgroup with the value weights staged in LDS: 29.6 us per
// launch at 256 boards -- 64 workgroups, 64 KB staged by each.)
constexpr int kTailThreads = 256, kTailPer = 8;  // A <= 2048

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();  // red is reused by consecutive reductions
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < kTailThreads / 64; ++w) r = is_max ? fmaxf(r, red[w]) : r + red[w];
  return r;
}

// one board's softmax (in place over its logits) and value head; every
// thread of the 256 takes part (block reductions).  pre: chess's preloaded
// value weights wj (heads_tail_kernel)
__device__ __forceinline__ void tail_board(const float4* __restrict__ feat, const HeadWeights& hw, int HW, int A,
                                           int hidden, float* __restrict__ probs, float* __restrict__ values,
                                           int b, bool pre, const float (&wj)[64], float* vflat, float* red) {
  const int t = threadIdx.x;
  __syncthreads();  // vflat of the previous board is no longer read
  for (int p = t; p < HW; p += kTailThreads) vflat[p] = feat[(size_t)b * HW + p].z;
  float* row = probs + (size_t)b * A;
  float x[kTailPer];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < kTailPer; ++k) {
    const int a = t + k * kTailThreads;
    x[k] = a < A ? row[a] : -INFINITY;
    m = fmaxf(m, x[k]);
  }
  m = block_reduce(m, red, true);
  float z = 0.f;
#pragma unroll
  for (int k = 0; k < kTailPer; ++k) {
    const int a = t + k * kTailThreads;
    x[k] = a < A ? expf(x[k] - m) : 0.f;
    z += x[k];
  }
  z = block_reduce(z, red, false);  // its barriers also publish vflat
#pragma unroll
  for (int k = 0; k < kTailPer; ++k) {
    const int a = t + k * kTailThreads;
    if (a < A) row[a] = x[k] / z;
  }
  float part = 0.f;
  if (pre) {
    if (t < hidden) {
      float sv = hw.bv1[t];
#pragma unroll
      for (int p = 0; p < 64; ++p) sv += vflat[p] * wj[p];
      part += fmaxf(sv, 0.f) * hw.wv2[t];
    }
  } else {
    for (int j = t; j < hidden; j += kTailThreads) {
      float sv = hw.bv1[j];
#pragma unroll 16
      for (int p = 0; p < HW; ++p) sv += vflat[p] * hw.wv1[p * hidden + j];
      part += fmaxf(sv, 0.f) * hw.wv2[j];
    }
  }
  part = block_reduce(part, red, false);
  if (t == 0) values[b] = tanhf(part + hw.bv2[0]);
}

__device__ __forceinline__ bool tail_preload(const HeadWeights& hw, int HW, int hidden, float (&wj)[64]) {
  // chess (HW = 64, hidden <= 256): the thread's hidden unit's 64 value
  // weights are loaded once, all in flight together, under the softmax (the
  // loop awaited them 16 at a time after it) -- the same sums
  const bool pre = HW == 64 && hidden <= kTailThreads;
  if (pre && (int)threadIdx.x < hidden) {
#pragma unroll
    for (int p = 0; p < 64; ++p) wj[p] = hw.wv1[p * hidden + threadIdx.x];
  }
  return pre;
}

__global__ __launch_bounds__(kTailThreads) void heads_tail_kernel(const float4* __restrict__ feat, HeadWeights hw,
                                                                  const int* __restrict__ count, int n_static,
                                                                  int HW, int A, int hidden,
                                                                  float* __restrict__ probs,
                                                                  float* __restrict__ values) {
  __shared__ float vflat[kMaxCells];
  __shared__ float red[kTailThreads / 64];
  const int n = count ? *count : n_static;
  float wj[64];
  const bool pre = tail_preload(hw, HW, hidden, wj);
  for (int b = blockIdx.x; b < n; b += gridDim.x)  // block-uniform
    tail_board(feat, hw, HW, A, hidden, probs, values, b, pre, wj, vflat, red);
}

// --------------------------------------------------------------- launchers
static void launch_policy_dense(const float4* feat, const float* wt, const float* b, const int* count, int n_max,
                                int HW, int A, float* logits, hipStream_t s) {
  if (n_max <= 256)
    policy_dense_kernel<128, 2><<<dim3((A + 63) / 64, (n_max + 7) / 8), 256, 0, s>>>(feat, wt, b, count, n_max, HW, A,
                                                                                     logits);
  else
    policy_dense_kernel<128, 8><<<dim3((A + 63) / 64, (n_max + 31) / 32), 256, 0, s>>>(feat, wt, b, count, n_max, HW,
                                                                                       A, logits);
}

void launch_encode(const Board* boards, const int* count, int n_max, int HW, float* x,
                   hipStream_t s) {
  const int total = n_max * HW;
  if (total <= 0) return;
  encode_boards_kernel<<<(total + 255) / 256, 256, 0, s>>>(boards, count, n_max, HW,
                                                           reinterpret_cast<float4*>(x));
}

void launch_legal_mask(const Board* boards, int n, const GameCfg& g, uint8_t* mask,
                       hipStream_t s) {
  const int total = n * g.A;
  if (total <= 0) return;
  legal_mask_kernel<<<(total + 255) / 256, 256, 0, s>>>(boards, n, g, mask);
}

// fp32 rows [n][c_src] -> [n][F] zero-padded: split16 (AZ_CONV_F16X2) or fp32 (AZ_CONV_DIRECT)
__global__ void pad_rows_kernel(const float* __restrict__ src, int n, int c_src, void* __restrict__ dst,
                                bool split) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * 32) return;
  const int r = idx >> 5, c4 = idx & 31;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * c4 + i;
    v[i] = c < c_src ? src[(size_t)r * c_src + c] : 0.f;
  }
  const float4 q = make_float4(v[0], v[1], v[2], v[3]);
  if (split) store_act4<true>(dst, (size_t)r, c4, q);
  else store_act4<false>(dst, (size_t)r, c4, q);
}

void launch_pad_rows(const float* src, int n, int c_src, void* dst, bool split, hipStream_t s) {
  if (n <= 0) return;
  pad_rows_kernel<<<(n * 32 + 255) / 256, 256, 0, s>>>(src, n, c_src, dst, split);
}

template <bool RES>
static void launch_direct(const float* in, const float* res_in, const float* w, const float* bias, float* out,
                          const int* count, int n_max, int H, int W, hipStream_t s) {
  const int grid = (n_max * H * W + 31) / 32;
  conv3x3_mfma_kernel<128, RES><<<grid, 256, conv_lds_bytes(32, W, RES), s>>>(
      in, res_in, reinterpret_cast<const float4*>(w), bias, out, count, n_max, H, W);
}

void launch_forward(const NetDev& net, const void* x, const int* count, int n_max, int H, int W,
                    int A, void* act_a, void* act_b, void* act_c, float* probs, float* values,
                    hipStream_t s, ConvTimer* timer, const Board* boards, int stem_first_chunk,
                    const TowerLeaves* leaves) {
  if (n_max <= 0) return;
  const int HW = H * W;
  constexpr int F = 128;
  const bool f16 = net.algo == AZ_CONV_F16X2;
  if (f16 && net.use_tower && net.in_ch == 4 && net.tower) {  // the whole forward in one launch
    if (timer) timer->begin(s);
    launch_tower16(net.tower, net.tower_rows, net.tower_alt_rows, net.tower_alt_staged, net.tower_staged, net.tower_dbuf, boards,
                   boards ? nullptr : static_cast<const float4*>(x), count, n_max, H, W, A, probs, values, net.err, s);
    if (timer) timer->end(s, 1);
    return;
  }
  if (f16 && net.use_tower && net.in_ch > 4 && net.tower && HW == 64 && A > kMaxActions) {
    // chess: the stem, the tower and the heads' 1x1 convs in one launch
    // (features into act_a), then the dense heads as below
    if (timer) timer->begin(s);
    launch_tower16_rows(net.tower, net.tower_rows, net.tower_staged, net.tower_dbuf, x, stem_first_chunk, count,
                        n_max, H, W, static_cast<float4*>(act_a), net.err, s, leaves);
    if (timer) timer->end(s, 1);
    HeadWeights hw{net.pc_w, net.pc_b, net.vc_w, net.vc_b, net.pd_w,
                   net.pd_b, net.v1_w, net.v1_b, net.v2_w, net.v2_b};
    const float4* feat = static_cast<const float4*>(act_a);
    launch_policy_dense(feat, net.pd_wt, net.pd_b, count, n_max, HW, A, probs, s);
    heads_tail_kernel<<<std::min(n_max, 2048), kTailThreads, 0, s>>>(feat, hw, count, n_max, HW, A, net.hidden, probs,
                                                                     values);
    return;
  }
  Conv16Args ca;
  ca.count = count;
  ca.n_max = n_max;
  ca.H = H;
  ca.W = W;
  // tile height by launch capacity: 32-row tiles for chess self-play's 256
  // boards, 48 for a lone launch of ~900 boards (profiles/micro/conv16_ab.sh),
  // 64 from ~1600 boards -- Connect-4 self-play lanes (2048 slots, ~870 live):
  // with the two lanes' convs sharing the CUs the larger tile's operand reuse
  // wins, 3207 vs 3137 games/s in-bench (profiles/r2/hw_queues.txt)
  const long rows_max = (long)n_max * HW;
  ca.mb = rows_max <= 24576 ? 2 : (rows_max <= 65536 ? 3 : 4);
  ca.err = net.err;
  if (net.in_ch > 4) {
    // chess: 118 input planes zero-padded to F, the stem is one more 3x3 conv;
    // stem_first_chunk: input chunks (32 planes) before it are known zero and
    // skipped -- they would add exact zeros (chess self-play: planes 0-63)
    if (f16) {
      Conv16Args a = ca;
      a.in = x;
      a.wpack = net.stem_k;
      a.bias = net.stem_b;
      a.oscale = net.stem_scale;
      a.out = act_a;
      a.first_chunk = stem_first_chunk;
      launch_conv16(a, s);
    } else {
      launch_direct<false>(static_cast<const float*>(x), nullptr, net.stem_d, net.stem_b,
                           static_cast<float*>(act_a), count, n_max, H, W, s);
    }
  } else {
    const int total = n_max * HW * (F / 4);
    if (boards) {
      if (f16)
        stem_board_kernel<F, true><<<std::min((n_max * HW + 7) / 8, 1024), 256, 0, s>>>(
            boards, net.stem_w, net.stem_b, count, n_max, H, W, act_a, net.err);
      else
        stem_board_kernel<F, false><<<std::min((n_max * HW + 7) / 8, 1024), 256, 0, s>>>(
            boards, net.stem_w, net.stem_b, count, n_max, H, W, act_a, nullptr);
    } else {
      const float4* x4 = static_cast<const float4*>(x);
      if (f16)
        stem_conv_kernel<F, true><<<(total + 255) / 256, 256, 0, s>>>(x4, net.stem_w, net.stem_b, count, n_max,
                                                                      H, W, act_a, net.err);
      else
        stem_conv_kernel<F, false><<<(total + 255) / 256, 256, 0, s>>>(x4, net.stem_w, net.stem_b, count, n_max,
                                                                       H, W, act_a, nullptr);
    }
  }
  void* cur = act_a;  // block input
  void* mid = act_b;
  void* nxt = act_c;
  if (timer) timer->begin(s);
  for (int d = 0; d < net.depth; ++d) {
    const bool last = d == net.depth - 1;
    if (f16) {
      Conv16Args a = ca;
      a.in = cur;
      a.wpack = net.k1[d];
      a.bias = net.c1_b[d];
      a.oscale = net.k1_scale[d];
      a.out = mid;
      launch_conv16(a, s);
      // the last block's conv2 runs the heads' 1x1 convs in its epilogue:
      // features [rows] float4 into nxt instead of the block output
      Conv16Args b = ca;
      b.in = mid;
      b.res_in = cur;
      b.wpack = net.k2[d];
      b.bias = net.c2_b[d];
      b.oscale = net.k2_scale[d];
      b.out = nxt;
      if (last) b.heads = Conv16Heads{net.pc_w, net.pc_b, net.vc_w, net.vc_b, static_cast<float4*>(nxt)};
      launch_conv16(b, s);
    } else {
      launch_direct<false>(static_cast<const float*>(cur), nullptr, net.c1_w[d], net.c1_b[d],
                           static_cast<float*>(mid), count, n_max, H, W, s);
      launch_direct<true>(static_cast<const float*>(mid), static_cast<const float*>(cur), net.c2_w[d],
                          net.c2_b[d], static_cast<float*>(nxt), count, n_max, H, W, s);
    }
    void* t = cur;
    cur = nxt;
    nxt = t;
  }
  if (timer) timer->end(s, 2 * net.depth);
  const float* act = static_cast<const float*>(cur);  // f16: the fused head features; direct: block output
  HeadWeights hw{net.pc_w, net.pc_b, net.vc_w, net.vc_b, net.pd_w,
                 net.pd_b, net.v1_w, net.v1_b, net.v2_w, net.v2_b};
  const size_t wbytes = (size_t)(2 * HW * A + HW * net.hidden) * sizeof(float);
  const bool stage = wbytes <= 64 * 1024;
  const int hblocks = stage ? std::min((n_max + 3) / 4, 512) : (n_max + 3) / 4;
#define AZ_HEADS(FEAT_, STAGE_)                                                                      \
  heads_kernel<F, FEAT_, STAGE_, kMaxActions><<<hblocks, 256, STAGE_ ? wbytes : 0, s>>>(           \
      act, hw, count, n_max, HW, A, net.hidden, probs, values)
  if (A > kMaxActions) {  // chess: 1880 actions
    if (f16 && HW == 64 && A <= kTailThreads * kTailPer && net.pd_wt) {
      const float4* feat = reinterpret_cast<const float4*>(act);
      launch_policy_dense(feat, net.pd_wt, net.pd_b, count, n_max, HW, A, probs, s);
      heads_tail_kernel<<<std::min(n_max, 2048), kTailThreads, 0, s>>>(feat, hw, count, n_max, HW, A,
                                                                       net.hidden, probs, values);
    } else {
      heads_kernel<F, false, false, 2048><<<(n_max + 3) / 4, 256, 0, s>>>(act, hw, count, n_max, HW, A,
                                                                          net.hidden, probs, values);
    }
  } else if (f16) {
    if (stage) AZ_HEADS(true, true); else AZ_HEADS(true, false);
  } else {
    if (stage) AZ_HEADS(false, true); else AZ_HEADS(false, false);
  }
#undef AZ_HEADS
}

}  // namespace az
