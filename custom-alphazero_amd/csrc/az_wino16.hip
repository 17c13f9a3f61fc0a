// az_wino16.hip -- the residual tower's Winograd F(2x2,3x3) convolutions on
// v_mfma_f32_16x16x4_f32 with 16 tiles per workgroup: the small-launch
// variant of wino_conv_kernel (az_wino.hip).
//
// Same layer, same transforms, same LDS layout of V, same host-side U (packed
// in this kernel's fragment order, wino16_pack_index).  What changes is the
// work split: a workgroup owns 16 consecutive 2x2 tiles x 128 output channels
// (wave w: channels [32w, 32w+32) as two 16-wide MFMA N blocks), so each wave
// issues half the MFMA cycles of the 32-tile kernel and a launch has twice the
// workgroups.  At the batch sizes self-play runs (a lane's ~700 Connect-4
// boards = 263 workgroups of 32 tiles on 256 CUs; 256 chess boards = 128) the
// 32-tile kernel leaves one workgroup per CU and one wave per SIMD, so the
// MFMA chain of one wave is the launch's critical path; here it is half as
// long and the V buffer (40 KB) leaves room for three workgroups per CU.
// MFMA 16x16x4: A[m = lane%16][k = lane/16], B[k = lane/16][n = lane%16],
// D[m = 4*(lane/16) + v][n = lane%16].  A lane's k quarter g takes input
// channels 8g..8g+7 of the chunk (k-step s: channel 8g + s).  Reduction
// order per output: chunk, point, k-step -- batch invariant, different from
// the 32-tile kernel (an engine uses one variant for every forward).
#include "az_nn.h"

namespace az {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kW16Tiles = 16;
constexpr int kW16Threads = 256;
// minimum waves per SIMD for the register allocator: 2 gives 138 VGPRs and no
// spills (3 waves/SIMD by registers); 4 forces 128 VGPRs with 5-9 spilled
#ifndef AZ_W16_OCC
#define AZ_W16_OCC 2
#endif
// stages of B (weight fragments) in flight ahead of the MFMAs that use them:
// 2 measured best (chess 484k -> 585k expansions/s, C4 +2%; 3 = 2)
#ifndef AZ_W16_PF
#define AZ_W16_PF 2
#endif
// 1: the next chunk's patch loads are issued at the start of the current
// chunk's MFMA stages (latency hidden behind them; the patch stays in
// registers until the chunk ends).  Measured slower: 188 VGPRs drop the
// kernel to 2 waves/SIMD (B=4096 178 vs 185 TFLOP/s, C4 self-play -4%)
#ifndef AZ_W16_EARLY
#define AZ_W16_EARLY 0
#endif


__host__ __device__ constexpr int w16_sign(int a, int i) {
  return i == 0 ? (a == 3 ? 0 : 1) : (a == 0 ? 0 : (a == 1 ? 1 : -1));
}

template <int CK>
__device__ __forceinline__ int w16_swz(int j, int t) {
  constexpr int RC = CK / 4, RPB = 16 / RC;
  return j ^ ((t / RPB) & (RC - 1));
}

// V row (tile) that MFMA row m holds.  ds_read_b128 serves a wave in lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): each group mixes k
// quarters 0 and 1 (or 2 and 3) over complementary row sets, so rows 0-3 and
// 12-15 go to tiles 0-7 and rows 4-11 to tiles 8-15 -- with the XOR swizzle
// every group then reads 16 distinct bank slots (identity: 2-way conflicts).
__device__ __forceinline__ int w16_tile(int m) { return m < 4 ? m : (m < 12 ? m + 4 : m - 8); }

// NS = 2 splits the 128 output channels over two workgroups (blockIdx.y):
// wave w of half h owns the 16 channels 64h + 16w .. +15 (one N block), so a
// launch has twice the workgroups and each wave half the MFMA chain, at the
// cost of both halves building the same V.  For launches too small to fill
// the CUs (a chess step's 256 boards = 256 workgroups); the same reduction
// order per output, so both splits give identical results.
template <bool RESIDUAL, bool HEADS, int NS>
__global__ __launch_bounds__(kW16Threads, AZ_W16_OCC) void wino16_conv_kernel(
    const float* __restrict__ in, const float* __restrict__ res_in,
    const float4* __restrict__ upack, const float4* __restrict__ rpack,
    const float* __restrict__ bias, float* __restrict__ out, const int* __restrict__ count,
    int n_static, int H, int W, HeadConv hc, int c0) {
  constexpr int CK = 32;
  constexpr int NX = RESIDUAL ? 20 : 16;
  constexpr int RC = CK / 4;                 // float4 per V row
  constexpr int VB = NX * kW16Tiles * RC;    // float4 in the V buffer
  constexpr int NCH = 128 / CK;
  constexpr int KS = CK / 4;                 // k-steps per stage (lane quarter: 8 channels)
  static_assert(NS == 1 || (NS == 2 && !HEADS), "the fused heads need all 128 channels");
  constexpr int NBW = 2 / NS;                // N blocks (16 channels) per wave
  constexpr int QB = 2 * NBW;                // float4 of B per lane per stage (NBW N blocks x 8)
  constexpr int IPT = 2 * kW16Tiles * RC / kW16Threads;  // producer items per thread (1)
  static_assert(IPT == 1, "one producer item per thread");
  __shared__ float4 vbuf[VB];

  const int HW = H * W, TW = (W + 1) >> 1, TH = (H + 1) >> 1, TB = TH * TW;
  const int n_boards = count ? *count : n_static;
  const int tiles = n_boards * TB;
  const int t0 = blockIdx.x * kW16Tiles;
  if (t0 >= tiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- producer geometry: thread -> (4-channel group pc, half ph, tile pt);
  // the 8 lanes of a ds_write_b128 group store 8 distinct 16-B slots of a row
  const int pc = tid & (RC - 1), ph = (tid / RC) & 1, pt = tid / (2 * RC);
  const int tau_p = t0 + pt;
  const bool pvalid = tau_p < tiles;
  int pbase = pc * 4, pty = 0, ptx = 0;
  if (pvalid) {
    const int b = tau_p / TB, lt = tau_p - b * TB;
    pty = lt / TW;
    ptx = lt - pty * TW;
    pbase += b * HW * 128;
  }
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 d[3][4], rr[2];
  uint32_t ok = 0;
  auto produce_load = [&](int c) {
    const int cb = c * CK;
    ok = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int y = 2 * pty - 1 + ph + r;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int xx = 2 * ptx - 1 + x;
        const bool o = pvalid && y >= 0 && y < H && xx >= 0 && xx < W;
        const unsigned off = o ? (unsigned)(pbase + (y * W + xx) * 128 + cb) : 0u;
        d[r][x] = *reinterpret_cast<const float4*>(in + off);
        ok |= (uint32_t)o << (r * 4 + x);
      }
    }
    if constexpr (RESIDUAL) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int p = 2 * ph + k;
        const int y = 2 * pty + (p >> 1), xx = 2 * ptx + (p & 1);
        const bool o = pvalid && y < H && xx < W;
        const unsigned off = o ? (unsigned)(pbase + (y * W + xx) * 128 + cb) : 0u;
        rr[k] = *reinterpret_cast<const float4*>(res_in + off);
        ok |= (uint32_t)o << (12 + k);
      }
    }
  };
  auto produce_store = [&]() {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        if (!((ok >> (r * 4 + x)) & 1)) d[r][x] = z4;
    if constexpr (RESIDUAL) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (!((ok >> (12 + k)) & 1)) rr[k] = z4;
    }
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
    const int sw = w16_swz<CK>(pc, pt);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int i = 2 * ph + ii;
      const float4 q0 = T[ii][0], q1 = T[ii][1], q2 = T[ii][2], q3 = T[ii][3];
      const float4 v[4] = {make_float4(q0.x - q2.x, q0.y - q2.y, q0.z - q2.z, q0.w - q2.w),
                           make_float4(q1.x + q2.x, q1.y + q2.y, q1.z + q2.z, q1.w + q2.w),
                           make_float4(q2.x - q1.x, q2.y - q1.y, q2.z - q1.z, q2.w - q1.w),
                           make_float4(q1.x - q3.x, q1.y - q3.y, q1.z - q3.z, q1.w - q3.w)};
#pragma unroll
      for (int j = 0; j < 4; ++j) vbuf[((i * 4 + j) * kW16Tiles + pt) * RC + sw] = v[j];
    }
    if constexpr (RESIDUAL) {
#pragma unroll
      for (int k = 0; k < 2; ++k) vbuf[((16 + 2 * ph + k) * kW16Tiles + pt) * RC + sw] = rr[k];
    }
  };

  // ---- consumer geometry: lane -> tile row r, k quarter g
  const int r = lane & 15, g = lane >> 4;
  f32x4 Y[4][NBW];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) Y[p][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the packed U keeps the 2-block-per-wave order (wino16_pack_index): a
  // split wave reads its N block's two float4 (q = 2 nb + s/4) from the
  // owning unsplit wave's fragment
  const int wsrc = NS == 1 ? wave : 2 * blockIdx.y + (wave >> 1);
  const int qoff = NS == 1 ? 0 : 2 * (wave & 1);
  const unsigned blane = (unsigned)((wsrc * 4 + qoff) * 64 + lane);
  const int colbase = NS == 1 ? 32 * wave : 64 * blockIdx.y + 16 * wave;
  auto load_b = [&](int c, int xi, float4 (&dst)[QB]) {
    const bool res = RESIDUAL && xi >= 16;
    const float4* base = res ? rpack : upack;
    const unsigned o = blane + (unsigned)(res ? c * 4 * 64 * 4 : (c * 16 + xi) * 4 * 64 * 4);
#pragma unroll
    for (int q = 0; q < QB; ++q) dst[q] = base[o + q * 64];
  };
  const int rt = w16_tile(r);  // this lane's A row (tile)
  auto load_a = [&](int xi, float4 (&dst)[2]) {
    const float4* vrow = vbuf + (xi * kW16Tiles + rt) * RC;
#pragma unroll
    for (int q = 0; q < 2; ++q) dst[q] = vrow[w16_swz<CK>(2 * g + q, rt)];
  };
  auto scatter = [&](int xi, const f32x4 (&m)[NBW]) {
    const int a = xi >> 2, bb = xi & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int si = w16_sign(a, i);
      if (si == 0) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int sj = w16_sign(bb, j);
        if (sj == 0) continue;
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) {
          if (si * sj > 0) Y[2 * i + j][nb] += m[nb];
          else Y[2 * i + j][nb] -= m[nb];
        }
      }
    }
  };
  constexpr int PF = AZ_W16_PF;
  constexpr int NB = PF == 1 ? 2 : 4;  // B register buffers (>= PF + 1, divides NX)
  float4 bq[NB][QB], aq[2][2];
  f32x4 M[2][NBW];
  // stage k of the flat (chunk, point) sequence -> its B fragments
  auto load_b_flat = [&](int k, float4 (&dst)[QB]) {
    if (k < NCH * NX) load_b(k / NX, k % NX, dst);
  };

  // c0 > 0: the input's first c0 chunks are zero (they would only add exact
  // zeros); flat stage c*NX + xi keeps its B buffer for any c0 (NX % NB == 0)
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
      // flat stage c*NX + xi uses buffer (c*NX + xi) % NB; NX % NB == 0 keeps it static
      static_assert(NX % NB == 0, "buffer of a stage must not depend on the chunk");
      load_b_flat(c * NX + xi + PF, bq[(xi + PF) % NB]);
      if (xi + 1 < NX) load_a(xi + 1, aq[(xi + 1) & 1]);
      if (AZ_W16_EARLY && xi == 0 && c + 1 < NCH) produce_load(c + 1);
      float av[KS], bv[NBW][KS];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float4 a4 = aq[xi & 1][q];
        av[4 * q] = a4.x, av[4 * q + 1] = a4.y, av[4 * q + 2] = a4.z, av[4 * q + 3] = a4.w;
      }
#pragma unroll
      for (int q = 0; q < QB; ++q) {  // q = 2 nb + s / 4
        const float4 b4 = bq[xi % NB][q];
        const int nb = q >> 1, s0 = (q & 1) * 4;
        bv[nb][s0] = b4.x, bv[nb][s0 + 1] = b4.y, bv[nb][s0 + 2] = b4.z, bv[nb][s0 + 3] = b4.w;
      }
      if (RESIDUAL && xi >= 16) {
        const int p = xi - 16;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb)
            Y[p][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[nb][s], Y[p][nb], 0, 0, 0);
      } else {
        f32x4(&m)[NBW] = M[xi & 1];
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb)
          m[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[nb][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < KS; ++s)
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb)
            m[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[nb][s], m[nb], 0, 0, 0);
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
      if (!AZ_W16_EARLY) produce_load(c + 1);
      produce_store();
      __syncthreads();
    }
  }

  // ---- epilogue: D row m = 4g + v (tile w16_tile(m)), column = 32 wave + 16 nb + (lane & 15)
  if constexpr (HEADS) {
    static_assert(RESIDUAL, "heads fuse into the block's second conv");
    static_assert(64 * 129 * 4 <= VB * 16, "the transpose fits the V buffer");
    float* tb = reinterpret_cast<float*>(vbuf);
    __syncthreads();  // V no longer read
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int col = wave * 32 + nb * 16 + r;
      const float bcol = bias[col];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = w16_tile(4 * g + v);
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
      const int tau = t0 + w16_tile(4 * g + v);
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

// float index of weight (cin, cout) at point xi in this kernel's B stream:
// float4 (((c*16 + xi)*4 + wave)*4 + q)*64 + lane, element e, where
// cin = 32c + 8*(lane>>4) + 4*(q&1) + e and cout = 32 wave + 16*(q>>1) + (lane&15).
size_t wino16_pack_index(int xi, int cin, int cout) {
  const int c = cin / 32, rem = cin % 32, gq = rem / 8, s = rem % 8;
  const int w = cout / 32, nb = (cout % 32) / 16, n16 = cout % 16;
  const int lane = gq * 16 + n16, q = nb * 2 + s / 4, e = s % 4;
  return (((((size_t)c * 16 + xi) * 4 + w) * 4 + q) * 64 + lane) * 4 + e;
}

void launch_wino16_conv(const float* in, const float* res_in, const float* upack, const float* rpack,
                        const float* bias, float* out, const int* count, int n_max, int H, int W,
                        hipStream_t s, const HeadConv* heads, int first_chunk) {
  const int TB = ((H + 1) / 2) * ((W + 1) / 2);
  const int grid = (n_max * TB + kW16Tiles - 1) / kW16Tiles;
  if (grid <= 0) return;
  const float4* u = reinterpret_cast<const float4*>(upack);
  const float4* rp = reinterpret_cast<const float4*>(rpack);
  // split the output channels over two workgroups when a launch has fewer
  // workgroups than AZ_W16_SPLIT_BELOW (default 640: C4 at ~700 boards +5%,
  // chess at 256 +3%, C4 at 1000 boards -5% if split; profiles/ab_split.sh); 0 = never
  static const int split_below = [] {
    const char* v = getenv("AZ_W16_SPLIT_BELOW");
    return v ? atoi(v) : 640;
  }();
  const bool split = grid < split_below;
  HeadConv hc{};
  if (heads && heads->feat) {
    hc = *heads;
    wino16_conv_kernel<true, true, 1><<<grid, kW16Threads, 0, s>>>(in, res_in, u, rp, bias, out, count, n_max,
                                                                   H, W, hc, 0);
  } else if (res_in) {
    if (split)
      wino16_conv_kernel<true, false, 2><<<dim3(grid, 2), kW16Threads, 0, s>>>(in, res_in, u, rp, bias, out,
                                                                              count, n_max, H, W, hc, 0);
    else
      wino16_conv_kernel<true, false, 1><<<grid, kW16Threads, 0, s>>>(in, res_in, u, rp, bias, out, count,
                                                                      n_max, H, W, hc, 0);
  } else {
    if (split)
      wino16_conv_kernel<false, false, 2><<<dim3(grid, 2), kW16Threads, 0, s>>>(
          in, nullptr, u, nullptr, bias, out, count, n_max, H, W, hc, first_chunk);
    else
      wino16_conv_kernel<false, false, 1><<<grid, kW16Threads, 0, s>>>(in, nullptr, u, nullptr, bias, out,
                                                                       count, n_max, H, W, hc, first_chunk);
  }
}

}  // namespace az
