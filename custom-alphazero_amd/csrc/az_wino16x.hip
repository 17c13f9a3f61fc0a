// az_wino16x.hip -- the 16-tile Winograd convolution with fp32 products
// built from three bf16 terms per operand on v_mfma_f32_16x16x32_bf16.
//
// gfx950's bf16 MFMA issues 16x the FLOP/cycle of its fp32 MFMA.  Each
// fp32 operand x is split exactly into x0 + x1 + x2 (bf16 each, 24
// significant bits: x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)),
// and a.b is accumulated from the six products a_i b_j with i + j <= 2,
// smallest first (a2b0, a1b1, a0b2, a1b0, a0b1, a0b0): the dropped terms are
// ~2^-24 relative, fp32's own rounding level, so the layer stays within
// NET_TOL of the float64 restatement.  Six 16-cycle bf16 MFMAs replace eight
// 32-cycle fp32 ones per 32-channel k-step (2.7x fewer MFMA cycles).
//
// Same tile split, transforms and channel split (NS) as wino16_conv_kernel.
// V is split once by the producer into three bf16 planes in LDS (48 / 60 KB),
// U once on the host (wino16x_pack_index).  MFMA 16x16x32 bf16: lane l holds
// A[row l&15][k = 8(l>>4) + j] and B[k = 8(l>>4) + j][col l&15], j = 0..7; D as
// the fp32 form.  A row m is tile m; a V plane row is 64 B (4 slots of 16 B),
// slot x16_swz(g, t) keeps every ds_read_b128 lane group on distinct banks.
// Reduction order per output: chunk, point, term -- batch invariant.
#include "az_nn.h"

namespace az {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kXTiles = 16;
constexpr int kXThreads = 256;
#ifndef AZ_W16X_PF
#define AZ_W16X_PF 2  // stages of B fragments in flight ahead of their MFMAs
#endif
#ifndef AZ_W16X_OCC
#define AZ_W16X_OCC 2  // minimum waves per SIMD for the register allocator
#endif

__host__ __device__ constexpr int x_sign(int a, int i) {
  return i == 0 ? (a == 3 ? 0 : 1) : (a == 0 ? 0 : (a == 1 ? 1 : -1));
}

// slot of lane quarter g in tile t's 64-B V row: lane groups {0-3,12-15,
// 20-27}, {4-11,16-19,28-31} (+32) read tiles {0-3,12-15} of one quarter with
// tiles 4-11 of the next; g ^ f(t / 4), f = (0, 2, 3, 1), separates them
__device__ __forceinline__ int x16_swz(int g, int t) { return g ^ ((0x78 >> (2 * (t >> 2))) & 3); }

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// two fp32 -> packed bf16 (lo, hi), round to nearest even: one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t bf16_pk(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{lo, hi}), bf16x2));
}
// the three bf16 terms of four channels, as three pairs of packed words
__device__ __forceinline__ void split3(const float4 v, uint2 (&t)[3]) {
  float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint32_t p0 = bf16_pk(x[0], x[1]), p1 = bf16_pk(x[2], x[3]);
    t[k] = make_uint2(p0, p1);
    if (k < 2) {
      x[0] -= __uint_as_float(p0 << 16);
      x[1] -= __uint_as_float(p0 & 0xffff0000u);
      x[2] -= __uint_as_float(p1 << 16);
      x[3] -= __uint_as_float(p1 & 0xffff0000u);
    }
  }
}

template <bool RESIDUAL, bool HEADS, int NS>
__global__ __launch_bounds__(kXThreads, AZ_W16X_OCC) void wino16x_conv_kernel(
    const float* __restrict__ in, const float* __restrict__ res_in,
    const uint4* __restrict__ upack, const uint4* __restrict__ rpack,
    const float* __restrict__ bias, float* __restrict__ out, const int* __restrict__ count,
    int n_static, int H, int W, HeadConv hc, int c0) {
  static_assert(NS == 1 || (NS == 2 && !HEADS), "the fused heads need all 128 channels");
  constexpr int CK = 32;
  constexpr int NX = RESIDUAL ? 20 : 16;
  constexpr int ROW = 4;                        // uint4 slots per V plane row
  constexpr int PLANE = NX * kXTiles * ROW;     // uint4 per plane
  constexpr int NCH = 128 / CK;
  constexpr int NBW = 2 / NS;                   // N blocks (16 channels) per wave
  constexpr int QB = 3 * NBW;                   // uint4 of B per lane per stage
  __shared__ uint4 vbuf[3 * PLANE];

  const int HW = H * W, TW = (W + 1) >> 1, TH = (H + 1) >> 1, TB = TH * TW;
  const int n_boards = count ? *count : n_static;
  const int tiles = n_boards * TB;
  const int t0 = blockIdx.x * kXTiles;
  if (t0 >= tiles) return;  // block-uniform
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- producer: thread -> (4-channel group pc, half ph, tile pt), as wino16
  const int pc = tid & 7, ph = (tid >> 3) & 1, pt = tid >> 4;
  const int tau_p = t0 + pt;
  const bool pvalid = tau_p < tiles;
  int pbase = pc * 4, pty = 0, ptx = 0;
  if (pvalid) {
    const int b = tau_p / TB, lt = tau_p - b * TB;
    pty = lt / TW;
    ptx = lt - pty * TW;
    pbase += b * HW * 128;
  }
  // buffer loads: the byte offset of each input pixel is chunk invariant
  // (voffset, computed once), the chunk goes in soffset; an off-board or
  // past-the-end pixel gets kOOB, which the descriptor's range check reads as 0
  const int in_bytes = n_static * HW * 128 * 4;  // < 2^31 (launcher)
  const auto in_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, in_bytes, 0x00020000);
  const auto res_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)(RESIDUAL ? res_in : in), (short)0, in_bytes, 0x00020000);
  constexpr unsigned kOOB = 0x80000000u;
  unsigned voff[3][4], roff[2];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int y = 2 * pty - 1 + ph + r;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int xx = 2 * ptx - 1 + x;
      const bool o = pvalid && y >= 0 && y < H && xx >= 0 && xx < W;
      voff[r][x] = o ? (unsigned)(pbase + (y * W + xx) * 128) * 4u : kOOB;
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = 2 * ph + k;
    const int y = 2 * pty + (p >> 1), xx = 2 * ptx + (p & 1);
    const bool o = RESIDUAL && pvalid && y < H && xx < W;
    roff[k] = o ? (unsigned)(pbase + (y * W + xx) * 128) * 4u : kOOB;
  }
  float4 d[3][4], rr[2];
  auto produce_load = [&](int c) {
    const int sb = c * CK * 4;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        d[r][x] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rsrc, voff[r][x], sb, 0));
    if constexpr (RESIDUAL) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
        rr[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(res_rsrc, roff[k], sb, 0));
    }
  };
  // 8-byte unit of (plane, point xi, tile pt, channel group pc)
  uint2* v2 = reinterpret_cast<uint2*>(vbuf);
  const int wslot = x16_swz(pc >> 1, pt) * 2 + (pc & 1);
  auto put = [&](int xi, const float4 v) {
    uint2 t[3];
    split3(v, t);
#pragma unroll
    for (int k = 0; k < 3; ++k) v2[(k * PLANE + (xi * kXTiles + pt) * ROW) * 2 + wslot] = t[k];
  };
  auto produce_store = [&]() {
    // T = B^T d (rows), B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]
    float4 T[2][4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const float4 a = d[0][x], b = d[1][x], e = d[2][x];
      if (ph == 0) {
        T[0][x] = make_float4(a.x - e.x, a.y - e.y, a.z - e.z, a.w - e.w);
        T[1][x] = make_float4(b.x + e.x, b.y + e.y, b.z + e.z, b.w + e.w);
      } else {
        T[0][x] = make_float4(b.x - a.x, b.y - a.y, b.z - a.z, b.w - a.w);
        T[1][x] = make_float4(a.x - e.x, a.y - e.y, a.z - e.z, a.w - e.w);
      }
    }
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int i = 2 * ph + ii;
      const float4 q0 = T[ii][0], q1 = T[ii][1], q2 = T[ii][2], q3 = T[ii][3];
      put(i * 4 + 0, make_float4(q0.x - q2.x, q0.y - q2.y, q0.z - q2.z, q0.w - q2.w));
      put(i * 4 + 1, make_float4(q1.x + q2.x, q1.y + q2.y, q1.z + q2.z, q1.w + q2.w));
      put(i * 4 + 2, make_float4(q2.x - q1.x, q2.y - q1.y, q2.z - q1.z, q2.w - q1.w));
      put(i * 4 + 3, make_float4(q1.x - q3.x, q1.y - q3.y, q1.z - q3.z, q1.w - q3.w));
    }
    if constexpr (RESIDUAL) {
#pragma unroll
      for (int k = 0; k < 2; ++k) put(16 + 2 * ph + k, rr[k]);
    }
  };

  // ---- consumer: lane -> tile row r, k quarter g
  const int r = lane & 15, g = lane >> 4;
  f32x4 Y[4][NBW];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) Y[p][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // B: uint4 ((((c*16 + xi)*4 + wsrc)*2 + nb)*3 + term)*64 + lane (wino16x_pack_index);
  // a split wave reads its N block's three terms from the owning wave's fragment
  const int wsrc = NS == 1 ? wave : 2 * blockIdx.y + (wave >> 1);
  const int nb0 = NS == 1 ? 0 : (wave & 1);
  // (buffer loads: lane part in voffset, chunk and point in soffset)
  const unsigned blane = (unsigned)((wsrc * 2 + nb0) * 3 * 64 + lane) * 16u;
  const auto u_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)upack, (short)0, NCH * 16 * 4 * 2 * 3 * 64 * 16,
                                                        0x00020000);
  const auto r_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(RESIDUAL ? rpack : upack), (short)0,
                                                        NCH * 4 * 2 * 3 * 64 * 16, 0x00020000);
  auto load_b = [&](int c, int xi, uint4 (&dst)[QB]) {
    const bool res = RESIDUAL && xi >= 16;
    const int so = (res ? c * 4 * 2 * 3 * 64 : (c * 16 + xi) * 4 * 2 * 3 * 64) * 16;
#pragma unroll
    for (int q = 0; q < QB; ++q)
      dst[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(res ? r_rsrc : u_rsrc, blane,
                                                                              so + q * 64 * 16, 0));
  };
  const int aslot = x16_swz(g, r);
  auto load_a = [&](int xi, uint4 (&dst)[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) dst[k] = vbuf[k * PLANE + (xi * kXTiles + r) * ROW + aslot];
  };
  auto scatter = [&](int xi, const f32x4 (&m)[NBW]) {
    const int a = xi >> 2, bb = xi & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int si = x_sign(a, i);
      if (si == 0) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int sj = x_sign(bb, j);
        if (sj == 0) continue;
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) {
          if (si * sj > 0) Y[2 * i + j][nb] += m[nb];
          else Y[2 * i + j][nb] -= m[nb];
        }
      }
    }
  };
  // the six term products, smallest first, into acc
  auto six = [&](const uint4 (&a)[3], const uint4* b, f32x4 acc) -> f32x4 {
    const bf16x8 a0 = __builtin_bit_cast(bf16x8, a[0]), a1 = __builtin_bit_cast(bf16x8, a[1]),
                 a2 = __builtin_bit_cast(bf16x8, a[2]);
    const bf16x8 b0 = __builtin_bit_cast(bf16x8, b[0]), b1 = __builtin_bit_cast(bf16x8, b[1]),
                 b2 = __builtin_bit_cast(bf16x8, b[2]);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b2, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
    return acc;
  };
  constexpr int PF = AZ_W16X_PF;
  constexpr int NB = PF == 1 ? 2 : 4;  // B register buffers (>= PF + 1, divides NX)
  static_assert(NX % NB == 0, "buffer of a stage must not depend on the chunk");
  uint4 bq[NB][QB], aq[2][3];
  f32x4 M[2][NBW];
  auto load_b_flat = [&](int k, uint4 (&dst)[QB]) {
    if (k < NCH * NX) load_b(k / NX, k % NX, dst);
  };

  produce_load(c0);
  produce_store();
#pragma unroll
  for (int k = 0; k < PF; ++k) load_b_flat(c0 * NX + k, bq[k]);
  __syncthreads();

#pragma unroll 1
  for (int c = c0; c < NCH; ++c) {
    load_a(0, aq[0]);
#pragma unroll
    for (int xi = 0; xi < NX; ++xi) {
      __builtin_amdgcn_sched_barrier(0);
      load_b_flat(c * NX + xi + PF, bq[(xi + PF) % NB]);
      if (xi + 1 < NX) load_a(xi + 1, aq[(xi + 1) & 1]);
      if (RESIDUAL && xi >= 16) {
        const int p = xi - 16;
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) Y[p][nb] = six(aq[xi & 1], &bq[xi % NB][3 * nb], Y[p][nb]);
      } else {
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb)
          M[xi & 1][nb] = six(aq[xi & 1], &bq[xi % NB][3 * nb], f32x4{0.f, 0.f, 0.f, 0.f});
      }
      if (xi >= 1 && xi - 1 < 16) {
        scatter(xi - 1, M[(xi - 1) & 1]);
        if constexpr (NBW == 2)
          asm volatile("" ::"v"(Y[0][0]), "v"(Y[0][1]), "v"(Y[1][0]), "v"(Y[1][1]), "v"(Y[2][0]), "v"(Y[2][1]),
                       "v"(Y[3][0]), "v"(Y[3][1]));
        else
          asm volatile("" ::"v"(Y[0][0]), "v"(Y[1][0]), "v"(Y[2][0]), "v"(Y[3][0]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (NX == 16) scatter(15, M[1]);
    if (c + 1 < NCH) {
      __syncthreads();
      produce_load(c + 1);
      produce_store();
      __syncthreads();
    }
  }

  // ---- epilogue: D row m = 4g + v (tile m), column = colbase + 16 nb + (lane & 15)
  const int colbase = NS == 1 ? 32 * wave : 64 * blockIdx.y + 16 * wave;
  if constexpr (HEADS) {
    static_assert(RESIDUAL, "heads fuse into the block's second conv");
    static_assert(64 * 129 * 4 <= 3 * PLANE * 16, "the transpose fits the V buffer");
    float* tb = reinterpret_cast<float*>(vbuf);
    __syncthreads();  // V no longer read
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int col = colbase + nb * 16 + r;
      const float bcol = bias[col];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = 4 * g + v;
#pragma unroll
        for (int p = 0; p < 4; ++p) tb[(row * 4 + p) * 129 + col] = fmaxf(Y[p][nb][v] + bcol, 0.0f);
      }
    }
    __syncthreads();
    if (tid < 64) {
      const int tau = t0 + (tid >> 2), p = tid & 3;
      if (tau < tiles) {
        const int b = tau / TB, lt = tau - b * TB;
        const int ty = lt / TW, tx = lt - ty * TW;
        const int y = 2 * ty + (p >> 1), x = 2 * tx + (p & 1);
        if (y < H && x < W) {
          const float* v = tb + tid * 129;
          float s0 = 0.f, s1 = 0.f, s2 = 0.f;
          for (int c = 0; c < 128; ++c) {
            s0 = fmaf(v[c], hc.wpc[2 * c], s0);
            s1 = fmaf(v[c], hc.wpc[2 * c + 1], s1);
            s2 = fmaf(v[c], hc.wvc[c], s2);
          }
          hc.feat[b * HW + y * W + x] = make_float4(fmaxf(s0 + hc.bpc[0], 0.f), fmaxf(s1 + hc.bpc[1], 0.f),
                                                    fmaxf(s2 + hc.bvc[0], 0.f), 0.f);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) {
    const int col = colbase + nb * 16 + r;
    const float bcol = bias[col];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int tau = t0 + 4 * g + v;
      if (tau >= tiles) continue;
      const int b = tau / TB, lt = tau - b * TB;
      const int ty = lt / TW, tx = lt - ty * TW;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int y = 2 * ty + (p >> 1), x = 2 * tx + (p & 1);
        if (y < H && x < W) out[(size_t)(b * HW + y * W + x) * 128 + col] = fmaxf(Y[p][nb][v] + bcol, 0.0f);
      }
    }
  }
}

// bf16 index (in 16-bit units) of term k of weight (cin, cout) at point xi:
// uint4 ((((c*16 + xi)*4 + w)*2 + nb)*3 + k)*64 + lane, element j, with
// cin = 32c + 8(lane>>4) + j and cout = 32w + 16nb + (lane&15)
size_t wino16x_pack_index(int xi, int cin, int cout, int k) {
  const int c = cin / 32, rem = cin % 32, gq = rem / 8, j = rem % 8;
  const int w = cout / 32, nb = (cout % 32) / 16, n16 = cout % 16;
  const int lane = gq * 16 + n16;
  return ((((((size_t)c * 16 + xi) * 4 + w) * 2 + nb) * 3 + k) * 64 + lane) * 8 + j;
}
// the 1x1 projection residual: one point per chunk
size_t wino16x_res_index(int cin, int cout, int k) {
  const int c = cin / 32, rem = cin % 32, gq = rem / 8, j = rem % 8;
  const int w = cout / 32, nb = (cout % 32) / 16, n16 = cout % 16;
  const int lane = gq * 16 + n16;
  return (((((size_t)c * 4 + w) * 2 + nb) * 3 + k) * 64 + lane) * 8 + j;
}

void launch_wino16x_conv(const float* in, const float* res_in, const float* upack, const float* rpack,
                         const float* bias, float* out, const int* count, int n_max, int H, int W,
                         hipStream_t s, const HeadConv* heads, int first_chunk) {
  const int TB = ((H + 1) / 2) * ((W + 1) / 2);
  const int grid = (n_max * TB + kXTiles - 1) / kXTiles;
  if (grid <= 0) return;
  const uint4* u = reinterpret_cast<const uint4*>(upack);
  const uint4* rp = reinterpret_cast<const uint4*>(rpack);
  static const int split_below = [] {
    const char* v = getenv("AZ_W16_SPLIT_BELOW");
    return v ? atoi(v) : 640;
  }();
  const bool split = grid < split_below;
  HeadConv hc{};
  if (heads && heads->feat) {
    hc = *heads;
    wino16x_conv_kernel<true, true, 1><<<grid, kXThreads, 0, s>>>(in, res_in, u, rp, bias, out, count, n_max,
                                                                  H, W, hc, 0);
  } else if (res_in) {
    if (split)
      wino16x_conv_kernel<true, false, 2><<<dim3(grid, 2), kXThreads, 0, s>>>(in, res_in, u, rp, bias, out,
                                                                             count, n_max, H, W, hc, 0);
    else
      wino16x_conv_kernel<true, false, 1><<<grid, kXThreads, 0, s>>>(in, res_in, u, rp, bias, out, count,
                                                                     n_max, H, W, hc, 0);
  } else {
    if (split)
      wino16x_conv_kernel<false, false, 2><<<dim3(grid, 2), kXThreads, 0, s>>>(
          in, nullptr, u, nullptr, bias, out, count, n_max, H, W, hc, first_chunk);
    else
      wino16x_conv_kernel<false, false, 1><<<grid, kXThreads, 0, s>>>(in, nullptr, u, nullptr, bias, out,
                                                                      count, n_max, H, W, hc, first_chunk);
  }
}

}  // namespace az
