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
//   stem_conv        K = 36, VALU
//   conv3x3_mfma     implicit GEMM on v_mfma_f32_32x32x2_f32 (exact f32 FMA
//                    chains): M = boards*HW rows, N = F, K = 9F (+F for the
//                    fused 1x1 projection residual).  MFMA bound.
//   heads            one wave per board
// Reduction order is fixed per output element and independent of the batch,
// so a board's outputs do not depend on what else is in the batch.
#include "az_nn.h"

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
template <int F>
__global__ __launch_bounds__(256) void stem_conv_kernel(const float4* __restrict__ x,
                                                        const float* __restrict__ ws,
                                                        const float* __restrict__ bias,
                                                        const int* __restrict__ count, int n_static,
                                                        int H, int W, float* __restrict__ out) {
  constexpr int G4 = F / 4;
  __shared__ float w_s[36 * F];
  for (int i = threadIdx.x; i < 36 * F; i += blockDim.x) w_s[i] = ws[i];
  __syncthreads();
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
      const float4 wv = *reinterpret_cast<const float4*>(w_s + (tap * 4 + c) * F + cg * 4);
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
  *reinterpret_cast<float4*>(out + (size_t)r * F + cg * 4) = acc;
}

// ------------------------------------------------------------ conv3x3 MFMA
// out[r][n] = ReLU( sum_k A[r][k] * wt[n][k] + bias[n] )
//   k in [0, 9F): A = in[neighbour(r, tap)][c], tap = k / F, c = k % F
//   k in [9F, 10F) (RESIDUAL): A = res_in[r][c]  (fused 1x1 projection)
// Tile: 128 rows x F=128 columns per 256-thread workgroup; wave w owns rows
// [32w, 32w+32) and all four 32-column MFMA tiles (64 accumulator VGPRs).
// K is consumed in chunks of 32 through a double-buffered LDS stage (A and B
// both [128][32] f32, rows padded to 36 floats: conflict-free ds_read_b128).
// Inside a chunk, lane half h owns k = 16h .. 16h+15, so MFMA k-step s sums
// the pair (s, 16+s): fixed order, batch-independent.
constexpr int kBM = 128;
constexpr int kKC = 32;
constexpr int kLdsStride = 36;  // floats per staged row (32 + 4 pad)

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int F, bool RESIDUAL>
__global__ __launch_bounds__(256, 2) void conv3x3_mfma_kernel(
    const float* __restrict__ in, const float* __restrict__ res_in, const float* __restrict__ wt,
    const float* __restrict__ bias, float* __restrict__ out, const int* __restrict__ count,
    int n_static, int H, int W) {
  static_assert(F == 128, "tile assumes F = 128 output channels");
  constexpr int K = (RESIDUAL ? 10 : 9) * F;
  constexpr int CPT = F / kKC;  // chunks per tap
  constexpr int NCHUNK = K / kKC;
  __shared__ __attribute__((aligned(16))) float lds[2][2][kBM * kLdsStride];  // [buf][A/B]

  const int HW = H * W;
  const int n_boards = count ? *count : n_static;
  const int rows = n_boards * HW;
  const int row0 = blockIdx.x * kBM;
  if (row0 >= rows) return;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;

  // staging geometry: piece q = tid + 256*j  ->  tile row q>>3, 4-float segment q&7
  const int seg = tid & 7;
  int src_b[4], src_y[4], src_x[4];
  bool src_ok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = row0 + (tid >> 3) + 32 * j;
    src_ok[j] = r < rows;
    const int b = r / HW, p = r - b * HW;
    src_b[j] = b;
    src_y[j] = p / W;
    src_x[j] = p - (p / W) * W;
  }

  float4 sa[4], sb[4];
  auto load_chunk = [&](int c) {
    const int tap = c / CPT;
    const int c0 = (c - tap * CPT) * kKC + seg * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (src_ok[j]) {
        if (tap < 9) {
          const int ny = src_y[j] + tap / 3 - 1, nx = src_x[j] + tap % 3 - 1;
          if (ny >= 0 && ny < H && nx >= 0 && nx < W)
            v = *reinterpret_cast<const float4*>(in + ((size_t)(src_b[j] * HW + ny * W + nx)) * F + c0);
        } else {
          v = *reinterpret_cast<const float4*>(
              res_in + ((size_t)(src_b[j] * HW + src_y[j] * W + src_x[j])) * F + c0);
        }
      }
      sa[j] = v;
      const int n = (tid >> 3) + 32 * j;
      sb[j] = *reinterpret_cast<const float4*>(wt + (size_t)n * K + c * kKC + seg * 4);
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = (tid >> 3) + 32 * j;
      *reinterpret_cast<float4*>(&lds[buf][0][row * kLdsStride + seg * 4]) = sa[j];
      *reinterpret_cast<float4*>(&lds[buf][1][row * kLdsStride + seg * 4]) = sb[j];
    }
  };

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.0f;

  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  for (int c = 0; c < NCHUNK; ++c) {
    const int buf = c & 1;
    if (c + 1 < NCHUNK) load_chunk(c + 1);
    const float* As = &lds[buf][0][(wave * 32 + r32) * kLdsStride + h * 16];
    float a[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(As + 4 * q);
      a[4 * q] = v.x;
      a[4 * q + 1] = v.y;
      a[4 * q + 2] = v.z;
      a[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float* Bs = &lds[buf][1][(t * 32 + r32) * kLdsStride + h * 16];
      float bv[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(Bs + 4 * q);
        bv[4 * q] = v.x;
        bv[4 * q + 1] = v.y;
        bv[4 * q + 2] = v.z;
        bv[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int s = 0; s < 16; ++s)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], bv[s], acc[t], 0, 0, 0);
    }
    if (c + 1 < NCHUNK) store_chunk(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C/D map col = lane&31, row = (i&3) + 8*(i>>2) + 4*h
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int col = t * 32 + r32;
    const float bcol = bias[col];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = row0 + wave * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (row < rows) out[(size_t)row * F + col] = fmaxf(acc[t][i] + bcol, 0.0f);
    }
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

template <int F>
__global__ __launch_bounds__(256) void heads_kernel(const float* __restrict__ act, HeadWeights hw,
                                                    const int* __restrict__ count, int n_static,
                                                    int HW, int A, int hidden,
                                                    float* __restrict__ probs,
                                                    float* __restrict__ values) {
  __shared__ float pflat[4][2 * kMaxCells];
  __shared__ float vflat[4][kMaxCells];
  __shared__ float logits[4][kMaxActions];
  const int n = count ? *count : n_static;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + wave;
  if (b >= n) return;  // wave-uniform; no block barrier below
  const float* base = act + (size_t)b * HW * F;
  for (int p = lane; p < HW; p += 64) {
    const float4* row = reinterpret_cast<const float4*>(base + (size_t)p * F);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll 8
    for (int q = 0; q < F / 4; ++q) {
      const float4 v = row[q];
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * q + e;
        s0 += vv[e] * hw.wpc[2 * c];
        s1 += vv[e] * hw.wpc[2 * c + 1];
        s2 += vv[e] * hw.wvc[c];
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
    for (int i = 0; i < 2 * HW; ++i) s += pflat[wave][i] * hw.wpd[i * A + a];
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
    for (int p = 0; p < HW; ++p) s += vflat[wave][p] * hw.wv1[p * hidden + j];
    part += fmaxf(s, 0.f) * hw.wv2[j];
  }
  part = wave_sum(part);
  if (lane == 0) values[b] = tanhf(part + hw.bv2[0]);
}

// --------------------------------------------------------------- launchers
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

void launch_forward(const NetDev& net, const float* x, const int* count, int n_max, int H, int W,
                    int A, float* act_a, float* act_b, float* act_c, float* probs, float* values,
                    hipStream_t s, ConvTimer* timer) {
  if (n_max <= 0) return;
  const int HW = H * W;
  constexpr int F = 128;
  {
    const int total = n_max * HW * (F / 4);
    stem_conv_kernel<F><<<(total + 255) / 256, 256, 0, s>>>(
        reinterpret_cast<const float4*>(x), net.stem_w, net.stem_b, count, n_max, H, W, act_a);
  }
  const int grid = (n_max * HW + kBM - 1) / kBM;
  float* cur = act_a;  // block input
  float* mid = act_b;
  float* nxt = act_c;
  if (timer) timer->begin(s);
  for (int d = 0; d < net.depth; ++d) {
    conv3x3_mfma_kernel<F, false><<<grid, 256, 0, s>>>(cur, nullptr, net.c1_w[d], net.c1_b[d],
                                                      mid, count, n_max, H, W);
    conv3x3_mfma_kernel<F, true><<<grid, 256, 0, s>>>(mid, cur, net.c2_w[d], net.c2_b[d], nxt,
                                                     count, n_max, H, W);
    float* t = cur;
    cur = nxt;
    nxt = t;
  }
  if (timer) timer->end(s, 2 * net.depth);
  HeadWeights hw{net.pc_w, net.pc_b, net.vc_w, net.vc_b, net.pd_w,
                 net.pd_b, net.v1_w, net.v1_b, net.v2_w, net.v2_b};
  heads_kernel<F><<<(n_max + 3) / 4, 256, 0, s>>>(cur, hw, count, n_max, HW, A, net.hidden, probs,
                                                 values);
}

}  // namespace az
