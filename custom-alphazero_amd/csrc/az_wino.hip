// az_wino.hip -- the residual tower's 3x3 convolutions as Winograd F(2x2,3x3)
// on the fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Same layer as conv3x3_mfma (az_nn.hip; Keras Conv2D 'same' + folded BN,
// base_layers.py:20-66), different algorithm: the board is cut into 2x2
// output tiles (TH x TW = ceil(H/2) x ceil(W/2) per board, 12 for 6x7), and
// for each tile
//     Y = A^T [ sum_cin (G g G^T)[xi] * (B^T d B)[xi] ] A,   xi in 4x4,
// i.e. 16 GEMMs [tiles x 128] x [128 x 128] per layer instead of 9 shifted
// ones over 4 pixels each: 16*12 = 192 vs 9*42 = 378 MFMA row-passes per 6x7
// board (1.97x fewer MFMA FLOP; 9x9: 400 vs 729).  All transforms are adds
// (input, output) or done once on the host in float64 (weights); the result
// stays within ~1e-7 relative of the float64 Keras restatement, like the
// direct kernel (tests/test_engine_gpu.py, NET_TOL = 1e-5).
//
// Workgroup = 4 waves = 32 consecutive tiles (one MFMA M block) x 128 output
// channels; wave w owns output channels [32w, 32w+32).  Input channels run in
// 8 chunks of 16:
//   * produce: the 256 threads turn the chunk's 4x4 input patches (read from
//     global/L2; a pixel is shared by up to four tiles) into V = B^T d B and
//     store V[xi][tile][16 cin] in LDS (plus, for the block's second conv, the
//     4 output pixels' block-input rows for the fused 1x1 projection residual);
//   * consume: per xi, 8 MFMAs accumulate M = V[xi] U[xi] over the chunk
//     (A from LDS, B = host-packed U fragments streamed from global two
//     points ahead), then M is added into the four output-pixel accumulators
//     with the +-1 coefficients of A^T (x) A^T.  The residual's four pixel
//     rows accumulate straight into their pixel's accumulator.
// Reduction order per output element is fixed (chunk, xi, k-step), so a
// board's outputs do not depend on the rest of the batch.
#include "az_nn.h"

namespace az {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWinoTiles = 32;   // tiles per workgroup (MFMA M)
constexpr int kWinoCK = 16;      // input channels per chunk
constexpr int kWinoChunks = 128 / kWinoCK;

// V rows are 16 floats = four 16-byte chunks; chunk j of tile row t lives at
// j ^ ((t >> 2) & 3) so the 16 rows a ds_read_b128 lane group touches fall on
// 16 distinct bank quads.
__device__ __forceinline__ int vswz(int j, int t) { return j ^ ((t >> 2) & 3); }

// PIPE 0: one V buffer, chunk c+1 loaded+transformed between two barriers.
// PIPE 1: two V buffers; chunk c+1's patch loads are issued a whole chunk
//         early into registers and transformed after chunk c's MFMAs: one
//         barrier per chunk, no exposed global latency.
template <bool RESIDUAL, int PIPE>
__global__ __launch_bounds__(256, 2) void wino_conv_kernel(
    const float* __restrict__ in, const float* __restrict__ res_in,
    const float4* __restrict__ upack, const float4* __restrict__ rpack,
    const float* __restrict__ bias, float* __restrict__ out, const int* __restrict__ count,
    int n_static, int H, int W) {
  constexpr int NX = RESIDUAL ? 20 : 16;  // 16 Winograd points (+4 residual pixel rows)
  constexpr int VB = NX * kWinoTiles * 4;  // float4 per V buffer
  __shared__ float4 vbuf_all[(PIPE ? 2 : 1) * VB];

  const int HW = H * W, TW = (W + 1) >> 1, TH = (H + 1) >> 1, TB = TH * TW;
  const int n_boards = count ? *count : n_static;
  const int tiles = n_boards * TB;
  const int t0 = blockIdx.x * kWinoTiles;
  if (t0 >= tiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- producer geometry: thread -> (tile pt, 4-channel group pc, half ph)
  const int pt = tid >> 3, pc = (tid >> 1) & 3, ph = tid & 1;
  const int ptau = t0 + pt;
  const bool pvalid = ptau < tiles;
  int pb = 0, pty = 0, ptx = 0;
  if (pvalid) {
    pb = ptau / TB;
    const int lt = ptau - pb * TB;
    pty = lt / TW;
    ptx = lt - pty * TW;
  }
  // rows of the 4x4 patch this half needs: V rows i = 2ph, 2ph+1 use d rows
  // {0,1,2} (ph = 0) or {1,2,3} (ph = 1)
  int doff[3][4];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int y = 2 * pty - 1 + ph + r;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int x = 2 * ptx - 1 + c;
      const bool ok = pvalid && y >= 0 && y < H && x >= 0 && x < W;
      doff[r][c] = ok ? ((pb * HW + y * W + x) * 128 + pc * 4) : -1;
    }
  }
  int roff[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = 2 * ph + k;
    const int y = 2 * pty + (p >> 1), x = 2 * ptx + (p & 1);
    roff[k] = (RESIDUAL && pvalid && y < H && x < W) ? ((pb * HW + y * W + x) * 128 + pc * 4) : -1;
  }
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  struct Patch {
    float4 d[3][4];
    float4 rr[2];
  };
  // unconditional loads (clamped address) + select: no branches, all 12-14
  // loads in flight together
  auto produce_load = [&](int c, Patch& P) {
    const int cb = c * kWinoCK;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        P.d[r][x] = *reinterpret_cast<const float4*>(in + (unsigned)(doff[r][x] >= 0 ? doff[r][x] + cb : 0));
    if constexpr (RESIDUAL) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
        P.rr[k] = *reinterpret_cast<const float4*>(res_in + (unsigned)(roff[k] >= 0 ? roff[k] + cb : 0));
    }
  };
  auto produce_store = [&](Patch& P, float4* vbuf) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        if (doff[r][x] < 0) P.d[r][x] = z4;
    if constexpr (RESIDUAL) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (roff[k] < 0) P.rr[k] = z4;
    }
    // T = B^T d (rows), B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]
    float4 T[2][4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const float4 a = P.d[0][x], b = P.d[1][x], e = P.d[2][x];
      if (ph == 0) {  // rows 0,1 from d rows 0,1,2
        T[0][x] = make_float4(a.x - e.x, a.y - e.y, a.z - e.z, a.w - e.w);
        T[1][x] = make_float4(b.x + e.x, b.y + e.y, b.z + e.z, b.w + e.w);
      } else {        // rows 2,3 from d rows 1,2,3 (a = d1, b = d2, e = d3)
        T[0][x] = make_float4(b.x - a.x, b.y - a.y, b.z - a.z, b.w - a.w);
        T[1][x] = make_float4(a.x - e.x, a.y - e.y, a.z - e.z, a.w - e.w);
      }
    }
    const int sw = vswz(pc, pt);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int i = 2 * ph + ii;
      const float4 t0_ = T[ii][0], t1 = T[ii][1], t2 = T[ii][2], t3 = T[ii][3];
      const float4 v[4] = {
          make_float4(t0_.x - t2.x, t0_.y - t2.y, t0_.z - t2.z, t0_.w - t2.w),
          make_float4(t1.x + t2.x, t1.y + t2.y, t1.z + t2.z, t1.w + t2.w),
          make_float4(t2.x - t1.x, t2.y - t1.y, t2.z - t1.z, t2.w - t1.w),
          make_float4(t1.x - t3.x, t1.y - t3.y, t1.z - t3.z, t1.w - t3.w)};
#pragma unroll
      for (int j = 0; j < 4; ++j) vbuf[((i * 4 + j) * kWinoTiles + pt) * 4 + sw] = v[j];
    }
    if constexpr (RESIDUAL) {
#pragma unroll
      for (int k = 0; k < 2; ++k) vbuf[((16 + 2 * ph + k) * kWinoTiles + pt) * 4 + sw] = P.rr[k];
    }
  };

  // ---- consumer geometry: lane -> tile row r, k half h; wave -> columns
  const int r = lane & 31, h = lane >> 5;
  f32x16 Y[4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int i = 0; i < 16; ++i) Y[p][i] = 0.0f;

  // B stream: point g = c*NX + xi; two float4 per point.  Four register
  // buffers, prefetch distance 2 (NX % 4 == 0 keeps the ring position static
  // inside the unrolled point loop).  32-bit offsets from the uniform base.
  const unsigned blane = (unsigned)(wave * 128 + lane);
  auto load_b = [&](int c, int xi, float4 (&dst)[2]) {
    const float4* base = (RESIDUAL && xi >= 16) ? rpack : upack;
    const unsigned o = blane + (unsigned)((RESIDUAL && xi >= 16) ? c * 512 : (c * 16 + xi) * 512);
    dst[0] = base[o];
    dst[1] = base[o + 64];
  };
  auto load_a = [&](const float4* vbuf, int xi, float4 (&dst)[2]) {
    const float4* vrow = vbuf + (xi * kWinoTiles + r) * 4;
    dst[0] = vrow[vswz(2 * h, r)];
    dst[1] = vrow[vswz(2 * h + 1, r)];
  };
  // Y[p] +-= M for the output pixels point xi feeds:
  // A^T = [[1,1,1,0],[0,1,-1,-1]] on both axes
  auto scatter = [&](int xi, const f32x16& m) {
    const int a = xi >> 2, bb = xi & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int si = i == 0 ? (a == 3 ? 0 : 1) : (a == 0 ? 0 : (a == 1 ? 1 : -1));
      if (si == 0) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int sj = j == 0 ? (bb == 3 ? 0 : 1) : (bb == 0 ? 0 : (bb == 1 ? 1 : -1));
        if (sj == 0) continue;
        if (si * sj > 0) {
          Y[2 * i + j] += m;
        } else {
          Y[2 * i + j] -= m;
        }
      }
    }
  };
  float4 bq[4][2], aq[2][2];
  f32x16 M[2];

  Patch P;
  produce_load(0, P);
  produce_store(P, vbuf_all);
  if (PIPE) produce_load(1, P);
  load_b(0, 0, bq[0]);
  load_b(0, 1, bq[1]);
  __syncthreads();

  for (int c = 0; c < kWinoChunks; ++c) {
    const float4* vbuf = vbuf_all + (PIPE ? (c & 1) * VB : 0);
    load_a(vbuf, 0, aq[0]);
#pragma unroll
    for (int xi = 0; xi < NX; ++xi) {
      // one software-pipeline stage per point: the scheduler may interleave
      // inside a stage (MFMAs of xi with the adds of xi-1) but not across
      __builtin_amdgcn_sched_barrier(0);
      {
        const int nx = xi + 2;
        if (nx < NX) {
          load_b(c, nx, bq[nx & 3]);
        } else if (c + 1 < kWinoChunks) {
          load_b(c + 1, nx - NX, bq[nx & 3]);
        }
      }
      if (xi + 1 < NX) load_a(vbuf, xi + 1, aq[(xi + 1) & 1]);
      const float4 a0 = aq[xi & 1][0], a1 = aq[xi & 1][1];
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float4 b0 = bq[xi & 3][0], b1 = bq[xi & 3][1];
      const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      if (RESIDUAL && xi >= 16) {
        // fused 1x1 projection residual: pixel p's own block-input row
        const int p = xi - 16;
#pragma unroll
        for (int s = 0; s < 8; ++s) Y[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], Y[p], 0, 0, 0);
      } else {
        f32x16& m = M[xi & 1];
        m = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0], bv[0], f32x16{}, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < 8; ++s) m = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], m, 0, 0, 0);
      }
      if (xi >= 1 && xi - 1 < 16) {
        scatter(xi - 1, M[(xi - 1) & 1]);
        // pin the adds to this stage (IR-level sinking would otherwise move
        // every point's adds to the loop latch and keep 16 M blocks live)
        asm volatile("" ::"v"(Y[0]), "v"(Y[1]), "v"(Y[2]), "v"(Y[3]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (NX == 16) scatter(15, M[1]);
    if (c + 1 < kWinoChunks) {
      if constexpr (PIPE) {
        // the other buffer was last read in chunk c-1, before the previous
        // barrier: safe to overwrite now
        produce_store(P, vbuf_all + ((c + 1) & 1) * VB);
        if (c + 2 < kWinoChunks) produce_load(c + 2, P);
        __syncthreads();
      } else {
        __syncthreads();  // every wave is done with chunk c's V
        produce_load(c + 1, P);
        produce_store(P, vbuf_all);
        __syncthreads();
      }
    }
  }

  // ---- epilogue: bias (+ residual bias, folded on the host), ReLU, store
  // C/D map: column = lane & 31, tile row = (i & 3) + 8*(i >> 2) + 4*h
  const int col = wave * 32 + r;
  const float bcol = bias[col];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int tau = t0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (tau >= tiles) continue;
    const int b = tau / TB, lt = tau - b * TB;
    const int ty = lt / TW, tx = lt - ty * TW;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int y = 2 * ty + (p >> 1), x = 2 * tx + (p & 1);
      if (y < H && x < W) out[(size_t)(b * HW + y * W + x) * 128 + col] = fmaxf(Y[p][i] + bcol, 0.0f);
    }
  }
}

void launch_wino_conv(const float* in, const float* res_in, const float* upack,
                      const float* rpack, const float* bias, float* out, const int* count,
                      int n_max, int H, int W, hipStream_t s, int pipe) {
  const int TB = ((H + 1) / 2) * ((W + 1) / 2);
  const int grid = (n_max * TB + kWinoTiles - 1) / kWinoTiles;
  if (grid <= 0) return;
  const float4* u = reinterpret_cast<const float4*>(upack);
  const float4* rp = reinterpret_cast<const float4*>(rpack);
  if (pipe) {
    if (res_in)
      wino_conv_kernel<true, 1><<<grid, 256, 0, s>>>(in, res_in, u, rp, bias, out, count, n_max, H, W);
    else
      wino_conv_kernel<false, 1><<<grid, 256, 0, s>>>(in, nullptr, u, nullptr, bias, out, count, n_max, H, W);
  } else {
    if (res_in)
      wino_conv_kernel<true, 0><<<grid, 256, 0, s>>>(in, res_in, u, rp, bias, out, count, n_max, H, W);
    else
      wino_conv_kernel<false, 0><<<grid, 256, 0, s>>>(in, nullptr, u, nullptr, bias, out, count, n_max, H, W);
  }
}

}  // namespace az
