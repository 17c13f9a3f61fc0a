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
// Workgroup = 4 waves = 32 consecutive tiles (one MFMA M block; tiles cross
// board boundaries freely) x 128 output channels; wave w owns output
// channels [32w, 32w+32).  Input channels run in chunks of CK:
//   * produce: the 256 threads turn the chunk's 4x4 input patches (read from
//     global/L2; a pixel is shared by up to four tiles) into V = B^T d B and
//     store V[xi][tile][CK] in LDS (plus, for the block's second conv, the 4
//     output pixels' block-input rows for the fused 1x1 projection residual);
//   * consume, one pipeline stage per point xi: CK/2 MFMAs accumulate
//     M = V[xi] U[xi] over the chunk (A from LDS, B = host-packed U fragments
//     streamed from global one stage ahead), and the previous stage's M is
//     added into the four output-pixel accumulators with the +-1
//     coefficients of A^T (x) A^T.  The residual's pixel rows accumulate
//     straight into their pixel.
// Reduction order per output element is fixed (chunk, xi, k-step), so a
// board's outputs do not depend on the rest of the batch.
//
// The A/B record behind these choices (chunk 32 single-buffered over chunk
// 16 double-buffered, warp-specialised producers, corner points straight
// into their pixel, explicit instruction groups, two M blocks per workgroup)
// is in DESIGN.md section 5; those variants lost and were removed.
#include "az_nn.h"

namespace az {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWinoTiles = 32;   // tiles per workgroup (MFMA M)
constexpr int kWinoThreads = 256;

#ifndef AZ_WINO_DIAG
#define AZ_WINO_DIAG 0  // timing experiments only (wrong outputs): 1 no B stream, 2 no
                        // producer after chunk 0, 3 no output-transform adds, 4 = 1+2+3
#endif

// A^T = [[1,1,1,0],[0,1,-1,-1]]: sign with which point coordinate a feeds
// output coordinate i (0 = not at all)
__host__ __device__ constexpr int wino_sign(int a, int i) {
  return i == 0 ? (a == 3 ? 0 : 1) : (a == 0 ? 0 : (a == 1 ? 1 : -1));
}

// V rows are CK floats = CK/4 16-byte chunks; chunk j of tile row t is
// stored at j ^ f(t) with f(t) = (t / rows-per-256B) mod (CK/4), so the 16
// rows a ds_read_b128 lane group touches fall on 16 distinct bank quads.
template <int CK>
__device__ __forceinline__ int vswz(int j, int t) {
  constexpr int RC = CK / 4, RPB = 16 / RC;
  return j ^ ((t / RPB) & (RC - 1));
}

// HEADS: the last block's conv2 also runs the heads' 1x1 convolutions in its
// epilogue (feat, az_nn.h HeadConv) and never writes the block output.
// (HIP's second launch-bounds argument is the minimum waves per SIMD: two,
// i.e. two workgroups per CU, which the V buffer's LDS also allows.)
// KSPLIT = 2 (small batches, the chess engine): two groups of 4 waves share
// the workgroup's 32 tiles, group g takes input-channel chunks g, g+2 (each
// group its own V buffer), and group 1's accumulators are added into group
// 0's through LDS before the epilogue.  Each wave issues half the MFMAs, and
// with one workgroup per CU the 8 waves overlap one group's transform with
// the other's MFMAs.  The reduction order differs from KSPLIT = 1 (same
// layer, within NET_TOL), so an engine uses one variant for every forward.
template <bool RESIDUAL, int CK, bool HEADS, int KSPLIT>
__global__ __launch_bounds__(kWinoThreads * KSPLIT, KSPLIT == 1 ? 2 : 1) void wino_conv_kernel(
    const float* __restrict__ in, const float* __restrict__ res_in,
    const float4* __restrict__ upack, const float4* __restrict__ rpack,
    const float* __restrict__ bias, float* __restrict__ out, const int* __restrict__ count,
    int n_static, int H, int W, HeadConv hc) {
  static_assert(CK == 16 || CK == 32, "chunk of 16 or 32 input channels");
  static_assert(KSPLIT == 1 || KSPLIT == 2, "one or two chunk groups");
  constexpr int NX = RESIDUAL ? 20 : 16;   // 16 Winograd points (+4 residual pixel rows)
  constexpr int RC = CK / 4;               // float4 per V row
  constexpr int VB = NX * kWinoTiles * RC; // float4 in the V buffer
  constexpr int NCH = 128 / CK;
  constexpr int KS = CK / 2;               // MFMA k-steps per stage
  constexpr int QB = CK / 8;               // float4 of B (and of A) per lane per stage
  constexpr int IPT = 16 * CK / kWinoThreads;  // producer items per thread (tile, c4, half)
  __shared__ float4 vbuf_all[VB * KSPLIT];

  const int HW = H * W, TW = (W + 1) >> 1, TH = (H + 1) >> 1, TB = TH * TW;
  const int n_boards = count ? *count : n_static;
  const int tiles = n_boards * TB;
  const int t0 = blockIdx.x * kWinoTiles;
  if (t0 >= tiles) return;
  // kg = chunk group; tid/wave below are within the group
  const int kg = KSPLIT == 1 ? 0 : (int)(threadIdx.x >> 8);
  const int tid = threadIdx.x & (kWinoThreads - 1), lane = tid & 63, wave = tid >> 6;
  float4* vbuf = vbuf_all + kg * VB;

  // ---- producer geometry: item -> (tile pt, 4-channel group pc, half ph)
  int pt[IPT], pc[IPT], ph[IPT], pbase[IPT], pty[IPT], ptx[IPT];
  bool pvalid[IPT];
#pragma unroll
  for (int it = 0; it < IPT; ++it) {
    const int item = tid + kWinoThreads * it;
    ph[it] = item & 1;
    pc[it] = (item >> 1) & (RC - 1);
    pt[it] = item / (2 * RC);
    const int tau = t0 + pt[it];
    pvalid[it] = tau < tiles;
    int b = 0, ty = 0, tx = 0;
    if (pvalid[it]) {
      b = tau / TB;
      const int lt = tau - b * TB;
      ty = lt / TW;
      tx = lt - ty * TW;
    }
    pbase[it] = b * HW * 128 + pc[it] * 4;
    pty[it] = ty;
    ptx[it] = tx;
  }
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  struct Patch {
    float4 d[IPT][3][4];
    float4 rr[IPT][2];
    uint32_t ok[IPT];  // bit r*4+x: patch pixel on the board; bits 12,13: residual rows
  };
  // V rows i = 2ph, 2ph+1 need patch rows {0,1,2} (ph = 0) or {1,2,3} (ph = 1).
  // Unconditional loads from a clamped address: no branches, every load of
  // the chunk in flight together; off-board pixels are zeroed in
  // produce_store (zeroing right after each load made it a stall: -15%).
  auto produce_load = [&](int c, Patch& P) {
    const int cb = c * CK;
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
      P.ok[it] = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int y = 2 * pty[it] - 1 + ph[it] + r;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const int xx = 2 * ptx[it] - 1 + x;
          const bool ok = pvalid[it] && y >= 0 && y < H && xx >= 0 && xx < W;
          const unsigned o = ok ? (unsigned)(pbase[it] + (y * W + xx) * 128 + cb) : 0u;
          P.d[it][r][x] = *reinterpret_cast<const float4*>(in + o);
          P.ok[it] |= (uint32_t)ok << (r * 4 + x);
        }
      }
      if constexpr (RESIDUAL) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int p = 2 * ph[it] + k;
          const int y = 2 * pty[it] + (p >> 1), xx = 2 * ptx[it] + (p & 1);
          const bool ok = pvalid[it] && y < H && xx < W;
          const unsigned o = ok ? (unsigned)(pbase[it] + (y * W + xx) * 128 + cb) : 0u;
          P.rr[it][k] = *reinterpret_cast<const float4*>(res_in + o);
          P.ok[it] |= (uint32_t)ok << (12 + k);
        }
      }
    }
  };
  auto produce_store = [&](Patch& P) {
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int x = 0; x < 4; ++x)
          if (!((P.ok[it] >> (r * 4 + x)) & 1)) P.d[it][r][x] = z4;
      if constexpr (RESIDUAL) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
          if (!((P.ok[it] >> (12 + k)) & 1)) P.rr[it][k] = z4;
      }
      // T = B^T d (rows), B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]
      float4 T[2][4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const float4 a = P.d[it][0][x], b = P.d[it][1][x], e = P.d[it][2][x];
        if (ph[it] == 0) {  // rows 0,1 from d rows 0,1,2
          T[0][x] = make_float4(a.x - e.x, a.y - e.y, a.z - e.z, a.w - e.w);
          T[1][x] = make_float4(b.x + e.x, b.y + e.y, b.z + e.z, b.w + e.w);
        } else {            // rows 2,3 from d rows 1,2,3 (a = d1, b = d2, e = d3)
          T[0][x] = make_float4(b.x - a.x, b.y - a.y, b.z - a.z, b.w - a.w);
          T[1][x] = make_float4(a.x - e.x, a.y - e.y, a.z - e.z, a.w - e.w);
        }
      }
      const int sw = vswz<CK>(pc[it], pt[it]);
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * ph[it] + ii;
        const float4 t0_ = T[ii][0], t1 = T[ii][1], t2 = T[ii][2], t3 = T[ii][3];
        const float4 v[4] = {
            make_float4(t0_.x - t2.x, t0_.y - t2.y, t0_.z - t2.z, t0_.w - t2.w),
            make_float4(t1.x + t2.x, t1.y + t2.y, t1.z + t2.z, t1.w + t2.w),
            make_float4(t2.x - t1.x, t2.y - t1.y, t2.z - t1.z, t2.w - t1.w),
            make_float4(t1.x - t3.x, t1.y - t3.y, t1.z - t3.z, t1.w - t3.w)};
#pragma unroll
        for (int j = 0; j < 4; ++j) vbuf[((i * 4 + j) * kWinoTiles + pt[it]) * RC + sw] = v[j];
      }
      if constexpr (RESIDUAL) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
          vbuf[((16 + 2 * ph[it] + k) * kWinoTiles + pt[it]) * RC + sw] = P.rr[it][k];
      }
    }
  };

  // ---- consumer geometry: lane -> tile row r, k half h; wave -> columns
  const int r = lane & 31, h = lane >> 5;
  f32x16 Y[4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int i = 0; i < 16; ++i) Y[p][i] = 0.0f;

  // B stream: QB float4 per lane per stage, two register buffers (one stage
  // ahead; NX is even, so the buffer of a stage is static).  32-bit offsets
  // from the uniform base.
  const unsigned blane = (unsigned)(wave * 64 * QB + lane);
  auto load_b = [&](int c, int xi, float4 (&dst)[QB]) {
    if ((AZ_WINO_DIAG == 1 || AZ_WINO_DIAG == 4) && (c > 0 || xi > 1)) return;
    const bool res = RESIDUAL && xi >= 16;
    const float4* base = res ? rpack : upack;
    const unsigned o = blane + (unsigned)(res ? c * 4 * 64 * QB : (c * 16 + xi) * 4 * 64 * QB);
#pragma unroll
    for (int q = 0; q < QB; ++q) dst[q] = base[o + q * 64];
  };
  auto load_a = [&](int xi, float4 (&dst)[QB]) {
    const float4* vrow = vbuf + (xi * kWinoTiles + r) * RC;
#pragma unroll
    for (int q = 0; q < QB; ++q) dst[q] = vrow[vswz<CK>(QB * h + q, r)];
  };
  auto scatter = [&](int xi, const f32x16& m) {
    if (AZ_WINO_DIAG == 3 || AZ_WINO_DIAG == 4) {
      Y[xi & 3] += m;
      return;
    }
    const int a = xi >> 2, bb = xi & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int si = wino_sign(a, i);
      if (si == 0) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int sj = wino_sign(bb, j);
        if (sj == 0) continue;
        if (si * sj > 0) {
          Y[2 * i + j] += m;
        } else {
          Y[2 * i + j] -= m;
        }
      }
    }
  };
  float4 bq[2][QB], aq[2][QB];
  f32x16 M[2];

  Patch P;
  produce_load(kg, P);
  produce_store(P);
  load_b(kg, 0, bq[0]);
  __syncthreads();

  // the chunk loop stays rolled: one copy of the 16-20 unrolled stages is
  // already ~10 KB of code
#pragma unroll 1
  for (int ci = 0; ci < NCH / KSPLIT; ++ci) {
    const int c = ci * KSPLIT + kg;
    const bool more = ci + 1 < NCH / KSPLIT;
    load_a(0, aq[0]);
#pragma unroll
    for (int xi = 0; xi < NX; ++xi) {
      // one software-pipeline stage per point: the scheduler may interleave
      // inside a stage (MFMAs of xi with the adds of xi-1 and the next
      // stage's loads) but not across
      __builtin_amdgcn_sched_barrier(0);
      if (xi + 1 < NX) {
        load_b(c, xi + 1, bq[(xi + 1) & 1]);
        load_a(xi + 1, aq[(xi + 1) & 1]);
      } else if (more) {
        load_b(c + KSPLIT, 0, bq[(xi + 1) & 1]);
      }
      float av[KS], bv[KS];
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const float4 a4 = aq[xi & 1][q], b4 = bq[xi & 1][q];
        av[4 * q] = a4.x, av[4 * q + 1] = a4.y, av[4 * q + 2] = a4.z, av[4 * q + 3] = a4.w;
        bv[4 * q] = b4.x, bv[4 * q + 1] = b4.y, bv[4 * q + 2] = b4.z, bv[4 * q + 3] = b4.w;
      }
      if (RESIDUAL && xi >= 16) {
        // fused 1x1 projection residual: pixel p's own block-input row
        const int p = xi - 16;
#pragma unroll
        for (int s = 0; s < KS; ++s) Y[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], Y[p], 0, 0, 0);
      } else {
        f32x16& m = M[xi & 1];
        m = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0], bv[0], f32x16{}, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < KS; ++s) m = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], m, 0, 0, 0);
      }
      if (xi >= 1 && xi - 1 < 16) {
        scatter(xi - 1, M[(xi - 1) & 1]);
        // pin the adds to this stage (IR-level sinking would otherwise move
        // every point's adds to the loop latch and keep all M blocks live)
        asm volatile("" ::"v"(Y[0]), "v"(Y[1]), "v"(Y[2]), "v"(Y[3]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (NX == 16) scatter(15, M[1]);
    if (more) {
      __syncthreads();  // every wave is done with chunk c's V
      if (AZ_WINO_DIAG != 2 && AZ_WINO_DIAG != 4) {
        produce_load(c + KSPLIT, P);
        produce_store(P);
      }
      __syncthreads();
    }
  }
  if constexpr (KSPLIT == 2) {
    // group 1's accumulators into group 0's: [p*16 + i][wave*64 + lane]
    // (consecutive lanes, consecutive words: conflict-free)
    float* red = reinterpret_cast<float*>(vbuf_all);
    __syncthreads();  // both groups are done with their V buffers
    if (kg == 1) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[(p * 16 + i) * kWinoThreads + tid] = Y[p][i];
    }
    __syncthreads();
    if (kg == 0) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int i = 0; i < 16; ++i) Y[p][i] += red[(p * 16 + i) * kWinoThreads + tid];
    }
    __syncthreads();  // `red` (the V buffers) is free again for the epilogue
  }

  // ---- epilogue: bias (+ residual bias, folded on the host), ReLU, store
  // C/D map: column = lane & 31, tile row = (i & 3) + 8*(i >> 2) + 4*h
  const int col = wave * 32 + r;
  const float bcol = bias[col];
  if constexpr (HEADS) {
    // fused head 1x1 convs: the block output goes through LDS (transposed to
    // [tile pixel][channel], row pitch 129 floats: conflict-free both ways)
    // and thread tp sums its pixel's 128 channels in channel order -- the
    // same fmaf chains as heads_kernel on a stored output
    static_assert(RESIDUAL, "heads fuse into the block's second conv");
    static_assert(64 * 129 * 4 <= VB * 16, "half the transpose fits the V buffer");
    float* tb = reinterpret_cast<float*>(vbuf);
    // two passes of 16 tile rows (64 tile pixels) each
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      __syncthreads();  // V (or the previous pass) no longer read
#pragma unroll
      for (int i = 8 * half; i < 8 * half + 8; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h - 16 * half;
#pragma unroll
        for (int p = 0; p < 4; ++p)
          if (kg == 0) tb[(row * 4 + p) * 129 + col] = fmaxf(Y[p][i] + bcol, 0.0f);
      }
      __syncthreads();
      if (kg == 0 && tid < 64) {
        const int tau = t0 + 16 * half + (tid >> 2), p = tid & 3;
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
    }
    return;
  }
  if (kg != 0) return;
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

// float index of weight (cin, cout) at point xi in the kernel's B stream:
// float4 (((c*16 + xi)*4 + nb)*QB + q)*64 + lane, element e, where
// cin = CK*c + (CK/2)*(lane>>5) + 4q + e and cout = 32nb + (lane&31).
size_t wino_pack_index(int xi, int cin, int cout) {
  constexpr int CK = kWinoCK, QB = CK / 8;
  const int c = cin / CK, rem = cin % CK, hh = rem / (CK / 2), k = rem % (CK / 2);
  const int q = k / 4, e = k % 4, nb = cout / 32, lane = 32 * hh + cout % 32;
  return (((((size_t)c * 16 + xi) * 4 + nb) * QB + q) * 64 + lane) * 4 + e;
}

void launch_wino_conv(const float* in, const float* res_in, const float* upack,
                      const float* rpack, const float* bias, float* out, const int* count,
                      int n_max, int H, int W, hipStream_t s, const HeadConv* heads, int ksplit) {
  const int TB = ((H + 1) / 2) * ((W + 1) / 2);
  const int grid = (n_max * TB + kWinoTiles - 1) / kWinoTiles;
  if (grid <= 0) return;
  const float4* u = reinterpret_cast<const float4*>(upack);
  const float4* rp = reinterpret_cast<const float4*>(rpack);
  constexpr int CK = kWinoCK;
  HeadConv hc{};
  const bool fuse = heads && heads->feat;
  if (fuse) hc = *heads;
#define AZ_WINO_LAUNCH(KS_)                                                                          \
  if (fuse)                                                                                         \
    wino_conv_kernel<true, CK, true, KS_><<<grid, kWinoThreads * KS_, 0, s>>>(in, res_in, u, rp, bias, \
                                                                          out, count, n_max, H, W, hc); \
  else if (res_in)                                                                                  \
    wino_conv_kernel<true, CK, false, KS_><<<grid, kWinoThreads * KS_, 0, s>>>(                      \
        in, res_in, u, rp, bias, out, count, n_max, H, W, hc);                                      \
  else                                                                                              \
    wino_conv_kernel<false, CK, false, KS_><<<grid, kWinoThreads * KS_, 0, s>>>(                     \
        in, nullptr, u, nullptr, bias, out, count, n_max, H, W, hc);
  if (ksplit == 2) {
    AZ_WINO_LAUNCH(2)
  } else {
    AZ_WINO_LAUNCH(1)
  }
#undef AZ_WINO_LAUNCH
}

}  // namespace az
