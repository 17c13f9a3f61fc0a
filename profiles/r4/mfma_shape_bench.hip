// Diagnostic microbenchmark (not product code): the tower's 3x3-conv K loop
// on a 128-row LDS tile, 8 waves (2 M halves x 4 N quarters), split16
// products (3 MFMAs per k-step), a streamed weight set of 8 convs x 36
// k32-steps x 16 KB from L2, in two MFMA shapes:
//   SHAPE 0: v_mfma_f32_16x16x32_f16, 4 16-row blocks x 2 16-channel blocks per wave (the product's loop)
//   SHAPE 1: v_mfma_f32_32x32x16_f16, 2 32-row blocks x 1 32-channel block per wave (same FLOPs, half the MFMAs)
// The same bytes move in both (LDS reads, weight loads); only the MFMA shape
// and count differ.  Prints us per launch, the clock (s_memtime /
// s_memrealtime of workgroup 0) and loop cycles per conv.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mfma_shape_bench mfma_shape_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int TR = 128, CONVS = 8;

__device__ unsigned long long g_clk[4];

template <int SHAPE, int FL = 0, int MBW0 = 4, int TU = 1>
__global__ __launch_bounds__(512, 1) void kbench(const uint4* __restrict__ w, float* __restrict__ out, int W) {
  extern __shared__ __attribute__((aligned(16))) uint4 act[];
  constexpr int PITCH = SHAPE == 0 ? 544 : 528;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, mh = (FL & 128) ? wave & 1 : wave >> 2,
            nq = (FL & 128) ? wave >> 1 : wave & 3;
  for (int i = tid; i < (TR + 16) * PITCH / 16; i += 512) {
    const unsigned v = (unsigned)(i * 2654435761u);
    act[i] = make_uint4(v & 0x3bff3bff, (v >> 3) & 0x3bff3bff, (v >> 7) & 0x3bff3bff, (v >> 11) & 0x3bff3bff);
  }
  __syncthreads();
  unsigned long long t0 = 0, r0 = 0;
  if (tid == 0 && blockIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, 0x7fffffff, 0x00020000);
  const char* actb = reinterpret_cast<const char*>(act);
  float sink = 0.f;
  if constexpr (SHAPE == 0 && (FL & 32)) {
    // term-major k-steps on a single-buffered ring: a block's t1 fragment is
    // re-read right after its term-0 products, its t0 fragment after its
    // term-2 products (the product kernel's register budget)
    constexpr int MBW = MBW0;
    f4 acc[MBW][2];
    for (int mb = 0; mb < MBW; ++mb) acc[mb][0] = acc[mb][1] = f4{0, 0, 0, 0};
    const int voff = ((nq * 2) * 2 * 64 + lane) * 16, gq = lane >> 4, r16 = lane & 15;
    for (int cv = 0; cv < CONVS; ++cv) {
      uint4 bq[4][4];
      constexpr int PF = (FL & 16) ? 2 : 1;
      uint4 aq[MBW][2];
      int ad[MBW], adn[MBW];
      auto load_b = [&](int ks, uint4(&d)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          d[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * 1024, (cv * 40 + ks) * 16384, 0));
      };
      auto tap_addr = [&](int t, int(&o)[MBW]) {
        const int sh = (t / 3 - 1) * W + (t % 3 - 1);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          int r = mh * 64 + mb * 16 + r16;
          asm volatile("" : "+v"(r));
          o[mb] = ((r + sh) & 127) * PITCH + gq * 16;
        }
      };
      load_b(0, bq[0]);
      if (PF == 2) load_b(1, bq[1]);
      tap_addr(0, ad);
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        aq[mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb]);
        aq[mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 256);
      }
#pragma unroll 1
      for (int t = 0; t < 9; ++t) {
        tap_addr(t < 8 ? t + 1 : t, adn);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          __builtin_amdgcn_sched_barrier(0);
          const int ks = 4 * t + c;
          if (ks + PF < 36) load_b(ks + PF, bq[(c + PF) & 3]);
          const int nc = (c + 1) & 3;
          const uint4(&b)[4] = bq[c];
          const h8 B0[2] = {__builtin_bit_cast(h8, b[0]), __builtin_bit_cast(h8, b[2])};
          const h8 B1[2] = {__builtin_bit_cast(h8, b[1]), __builtin_bit_cast(h8, b[3])};
          const bool more = ks + 1 < 36;
          if constexpr (FL & 64) __builtin_amdgcn_sched_group_barrier(0x0020, 4, 0);
          if constexpr (FL & 64) {
            // lagged: a block's fragment is re-read after the NEXT block's products of that pass
            const char* an = actb + (c == 3 ? 0 : 0);
            (void)an;
            auto rd1 = [&](int mb) { aq[mb][1] = *reinterpret_cast<const uint4*>(actb + (c == 3 ? adn[mb] : ad[mb]) + 64 * nc + 256); };
            auto rd0n = [&](int mb) { aq[mb][0] = *reinterpret_cast<const uint4*>(actb + (c == 3 ? adn[mb] : ad[mb]) + 64 * nc); };
#pragma unroll
            for (int mb = 0; mb < MBW; ++mb) {
              const h8 a1 = __builtin_bit_cast(h8, aq[mb][1]);
#pragma unroll
              for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a1, acc[mb][nb], 0, 0, 0);
              if (mb == 0 && ks > 0) aq[MBW - 1][0] = *reinterpret_cast<const uint4*>(actb + ad[MBW - 1] + 64 * c);
              if (mb >= 1 && more) rd1(mb - 1);
              __builtin_amdgcn_sched_group_barrier(0x0008, 2, 0);
              if ((mb == 0 && ks > 0) || (mb >= 1 && more)) __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
            }
#pragma unroll
            for (int mb = 0; mb < MBW; ++mb) {
              const h8 a0 = __builtin_bit_cast(h8, aq[mb][0]);
#pragma unroll
              for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B1[nb], a0, acc[mb][nb], 0, 0, 0);
              if (mb == 0 && more) rd1(MBW - 1);
              __builtin_amdgcn_sched_group_barrier(0x0008, 2, 0);
              if (mb == 0 && more) __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
            }
#pragma unroll
            for (int mb = 0; mb < MBW; ++mb) {
              const h8 a0 = __builtin_bit_cast(h8, aq[mb][0]);
#pragma unroll
              for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a0, acc[mb][nb], 0, 0, 0);
              if (mb >= 1 && more) rd0n(mb - 1);
              __builtin_amdgcn_sched_group_barrier(0x0008, 2, 0);
              if (mb >= 1 && more) __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
            }
          } else {
          // term 0: t1 x B0, then the t1 fragment's next read
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            const h8 a1 = __builtin_bit_cast(h8, aq[mb][1]);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a1, acc[mb][nb], 0, 0, 0);
            if (more) aq[mb][1] = *reinterpret_cast<const uint4*>(actb + (c == 3 ? adn[mb] : ad[mb]) + 64 * nc + 256);
          }
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            const h8 a0 = __builtin_bit_cast(h8, aq[mb][0]);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B1[nb], a0, acc[mb][nb], 0, 0, 0);
          }
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            const h8 a0 = __builtin_bit_cast(h8, aq[mb][0]);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a0, acc[mb][nb], 0, 0, 0);
            if (more) aq[mb][0] = *reinterpret_cast<const uint4*>(actb + (c == 3 ? adn[mb] : ad[mb]) + 64 * nc);
          }
          }
          if (c == 3) {
#pragma unroll
            for (int mb = 0; mb < MBW; ++mb) ad[mb] = adn[mb];
          }
          __builtin_amdgcn_sched_group_barrier(0x0020, 4, 0);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x0008, 2 * MBW, 0);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
          }
        }
      }
      __syncthreads();
    }
    for (int mb = 0; mb < MBW; ++mb)
      for (int nb = 0; nb < 2; ++nb) sink += acc[mb][nb][0] + acc[mb][nb][1] + acc[mb][nb][2] + acc[mb][nb][3];
  } else if constexpr (SHAPE == 0) {
    constexpr int MBW = MBW0;
    f4 acc[MBW][2];
    for (int mb = 0; mb < MBW; ++mb) acc[mb][0] = acc[mb][1] = f4{0, 0, 0, 0};
    const int voff = ((nq * 2) * 2 * 64 + lane) * 16, gq = lane >> 4, r16 = lane & 15;
    for (int cv = 0; cv < CONVS; ++cv) {
      constexpr int PFB = (FL & 512) ? 2 : 1, NBB = 2 * PFB;
      uint4 bq[NBB][4];
      uint4 aq[2][MBW][2];
      int ad[MBW];
      auto load_b = [&](int ks, uint4(&d)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          d[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * 1024, (cv * 40 + ks) * 16384, 0));
      };
      auto set_tap = [&](int t) {
        const int sh = (t / 3 - 1) * W + (t % 3 - 1);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          int r = mh * 64 + mb * 16 + r16;
          asm volatile("" : "+v"(r));
          ad[mb] = ((r + sh) & 127) * PITCH + gq * 16;
        }
      };
      load_b(0, bq[0]);
      if (PFB == 2) load_b(1, bq[1]);
      set_tap(0);
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        aq[0][mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb]);
        aq[0][mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 256);
      }
#pragma unroll TU
      for (int t = 0; t < 9; ++t) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          __builtin_amdgcn_sched_barrier(0);
          const int ks = 4 * t + c;
          if (!(FL & 1) && ks + PFB < 36) load_b(ks + PFB, bq[(c + PFB) % NBB]);
          const int nc = (c + 1) & 3;
          if (c == 3 && t < 8) set_tap(t + 1);
          const uint4(&b)[4] = bq[c % NBB];
          const h8 B0[2] = {__builtin_bit_cast(h8, b[0]), __builtin_bit_cast(h8, b[2])};
          const h8 B1[2] = {__builtin_bit_cast(h8, b[1]), __builtin_bit_cast(h8, b[3])};
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            const h8 a0 = __builtin_bit_cast(h8, aq[c & 1][mb][0]), a1 = __builtin_bit_cast(h8, aq[c & 1][mb][1]);
            if (FL & 8) {
              if (mb == MBW - 1) {
#pragma unroll
                for (int tm = 0; tm < 3; ++tm)
#pragma unroll
                  for (int m2 = 0; m2 < MBW; ++m2) {
                    const h8 x0 = __builtin_bit_cast(h8, aq[c & 1][m2][0]), x1 = __builtin_bit_cast(h8, aq[c & 1][m2][1]);
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb)
                      acc[m2][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(tm == 1 ? B1[nb] : B0[nb], tm == 0 ? x1 : x0, acc[m2][nb], 0, 0, 0);
                  }
              }
            } else if (FL & 4) {
#pragma unroll
              for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a1, acc[mb][nb], 0, 0, 0);
#pragma unroll
              for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B1[nb], a0, acc[mb][nb], 0, 0, 0);
#pragma unroll
              for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a0, acc[mb][nb], 0, 0, 0);
            } else {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a1, acc[mb][nb], 0, 0, 0);
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B1[nb], a0, acc[mb][nb], 0, 0, 0);
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a0, acc[mb][nb], 0, 0, 0);
            }
            }
            if (!(FL & 2) && ks + 1 < 36) {
              aq[(c + 1) & 1][mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 64 * nc);
              aq[(c + 1) & 1][mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 64 * nc + 256);
            }
          }
          if (!(FL & 3)) {
          __builtin_amdgcn_sched_group_barrier(0x0020, 4, 0);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 6, 0);
            __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
          }
          }
        }
      }
      __syncthreads();
    }
    for (int mb = 0; mb < MBW; ++mb)
      for (int nb = 0; nb < 2; ++nb) sink += acc[mb][nb][0] + acc[mb][nb][1] + acc[mb][nb][2] + acc[mb][nb][3];
  } else if constexpr (SHAPE == 3) {
    // M quarters x N halves: wave = 2 blocks of 16 rows x 4 N blocks (64
    // channels); the 4 waves of an N half load the same fragments and are all
    // the older (0-3) or all the younger (4-7) wave of their SIMD
    constexpr int MBW = 2, NBW = 4;
    const int mq = wave & 3, nh = wave >> 2;
    f4 acc[MBW][NBW];
    for (int mb = 0; mb < MBW; ++mb)
      for (int nb = 0; nb < NBW; ++nb) acc[mb][nb] = f4{0, 0, 0, 0};
    const int voff = ((nh * NBW) * 2 * 64 + lane) * 16, gq = lane >> 4, r16 = lane & 15;
    for (int cv = 0; cv < CONVS; ++cv) {
      uint4 bq[2][2 * NBW];
      uint4 aq[2][MBW][2];
      int ad[MBW];
      auto load_b = [&](int ks, uint4(&d)[2 * NBW]) {
#pragma unroll
        for (int q = 0; q < 2 * NBW; ++q)
          d[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * 1024, (cv * 40 + ks) * 16384, 0));
      };
      auto set_tap = [&](int t) {
        const int sh = (t / 3 - 1) * W + (t % 3 - 1);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          int r = mq * 32 + mb * 16 + r16;
          asm volatile("" : "+v"(r));
          ad[mb] = ((r + sh) & 127) * PITCH + gq * 16;
        }
      };
      load_b(0, bq[0]);
      set_tap(0);
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        aq[0][mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb]);
        aq[0][mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 256);
      }
#pragma unroll 1
      for (int t = 0; t < 9; ++t) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          __builtin_amdgcn_sched_barrier(0);
          const int ks = 4 * t + c;
          if (!(FL & 1) && ks + 1 < 36) load_b(ks + 1, bq[(c + 1) & 1]);
          const int nc = (c + 1) & 3;
          if (c == 3 && t < 8) set_tap(t + 1);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            const h8 a0 = __builtin_bit_cast(h8, aq[c & 1][mb][0]), a1 = __builtin_bit_cast(h8, aq[c & 1][mb][1]);
#pragma unroll
            for (int nb = 0; nb < NBW; ++nb) {
              const h8 B0 = __builtin_bit_cast(h8, bq[c & 1][2 * nb]), B1 = __builtin_bit_cast(h8, bq[c & 1][2 * nb + 1]);
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0, a1, acc[mb][nb], 0, 0, 0);
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B1, a0, acc[mb][nb], 0, 0, 0);
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0, a0, acc[mb][nb], 0, 0, 0);
            }
            if (!(FL & 2) && ks + 1 < 36) {
              aq[(c + 1) & 1][mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 64 * nc);
              aq[(c + 1) & 1][mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 64 * nc + 256);
            }
          }
          if (!(FL & 3)) {
          __builtin_amdgcn_sched_group_barrier(0x0020, 2 * NBW, 0);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 3 * NBW, 0);
            __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
          }
          }
        }
      }
      __syncthreads();
    }
    for (int mb = 0; mb < MBW; ++mb)
      for (int nb = 0; nb < NBW; ++nb) sink += acc[mb][nb][0] + acc[mb][nb][1] + acc[mb][nb][2] + acc[mb][nb][3];
  } else if constexpr (SHAPE == 2) {
    constexpr int MBW = 8;
    f4 acc[MBW];
    for (int mb = 0; mb < MBW; ++mb) acc[mb] = f4{0, 0, 0, 0};
    const int voff = (wave * 2 * 64 + lane) * 16, gq = lane >> 4, r16 = lane & 15;
    for (int cv = 0; cv < CONVS; ++cv) {
      uint4 bq[2][2];
      uint4 aq[2][MBW][2];
      int ad[MBW];
      auto load_b = [&](int ks, uint4(&d)[2]) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          d[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * 1024, (cv * 40 + ks) * 16384, 0));
      };
      auto set_tap = [&](int t) {
        const int sh = (t / 3 - 1) * W + (t % 3 - 1);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          int r = mb * 16 + r16;
          asm volatile("" : "+v"(r));
          ad[mb] = ((r + sh) & 127) * PITCH + gq * 16;
        }
      };
      load_b(0, bq[0]);
      set_tap(0);
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        aq[0][mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb]);
        aq[0][mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 256);
      }
#pragma unroll 1
      for (int t = 0; t < 9; ++t) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          __builtin_amdgcn_sched_barrier(0);
          const int ks = 4 * t + c;
          if (!(FL & 1) && ks + 1 < 36) load_b(ks + 1, bq[(c + 1) & 1]);
          const int nc = (c + 1) & 3;
          if (c == 3 && t < 8) set_tap(t + 1);
          const h8 B0 = __builtin_bit_cast(h8, bq[c & 1][0]), B1 = __builtin_bit_cast(h8, bq[c & 1][1]);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            const h8 a0 = __builtin_bit_cast(h8, aq[c & 1][mb][0]), a1 = __builtin_bit_cast(h8, aq[c & 1][mb][1]);
            acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0, a1, acc[mb], 0, 0, 0);
            acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B1, a0, acc[mb], 0, 0, 0);
            acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0, a0, acc[mb], 0, 0, 0);
            if (!(FL & 2) && ks + 1 < 36) {
              aq[(c + 1) & 1][mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 64 * nc);
              aq[(c + 1) & 1][mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 64 * nc + 256);
            }
          }
          if (!(FL & 3)) {
          __builtin_amdgcn_sched_group_barrier(0x0020, 2, 0);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 3, 0);
            __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
          }
          }
        }
      }
      __syncthreads();
    }
    for (int mb = 0; mb < MBW; ++mb) sink += acc[mb][0] + acc[mb][1] + acc[mb][2] + acc[mb][3];
  } else {
    constexpr int MBW = 2;
    f16v acc[MBW];
    for (int mb = 0; mb < MBW; ++mb)
      for (int i = 0; i < 16; ++i) acc[mb][i] = 0.f;
    // [k16-step][N quarter][term][lane] x 16 B: 8 KB per k16 step
    const int voff = (nq * 2 * 64 + lane) * 16, hh = lane >> 5, r32 = lane & 31;
    for (int cv = 0; cv < CONVS; ++cv) {
      uint4 bq[2][2];
      uint4 aq[2][MBW][2];
      int ad[MBW];
      auto load_b = [&](int ks, uint4(&d)[2]) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          d[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * 1024, (cv * 80 + ks) * 8192, 0));
      };
      auto set_tap = [&](int t) {
        const int sh = (t / 3 - 1) * W + (t % 3 - 1);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          int r = mh * 64 + mb * 32 + r32;
          asm volatile("" : "+v"(r));
          ad[mb] = ((r + sh) & 127) * PITCH + hh * 16;
        }
      };
      load_b(0, bq[0]);
      set_tap(0);
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        aq[0][mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb]);
        aq[0][mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 256);
      }
#pragma unroll 1
      for (int t = 0; t < 9; ++t) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          __builtin_amdgcn_sched_barrier(0);
          const int ks = 8 * t + c;
          if (ks + 1 < 72) load_b(ks + 1, bq[(c + 1) & 1]);
          const int nc = (c + 1) & 7;
          if (c == 7 && t < 8) set_tap(t + 1);
          const h8 B0 = __builtin_bit_cast(h8, bq[c & 1][0]), B1 = __builtin_bit_cast(h8, bq[c & 1][1]);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            const h8 a0 = __builtin_bit_cast(h8, aq[c & 1][mb][0]), a1 = __builtin_bit_cast(h8, aq[c & 1][mb][1]);
            acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(B0, a1, acc[mb], 0, 0, 0);
            acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(B1, a0, acc[mb], 0, 0, 0);
            acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(B0, a0, acc[mb], 0, 0, 0);
            if (ks + 1 < 72) {
              aq[(c + 1) & 1][mb][0] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 32 * nc);
              aq[(c + 1) & 1][mb][1] = *reinterpret_cast<const uint4*>(actb + ad[mb] + 32 * nc + 256);
            }
          }
          __builtin_amdgcn_sched_group_barrier(0x0020, 2, 0);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 3, 0);
            __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
          }
        }
      }
      __syncthreads();
    }
    for (int mb = 0; mb < MBW; ++mb)
      for (int i = 0; i < 16; ++i) sink += acc[mb][i];
  }
  if (tid == 0 && blockIdx.x == 0) {
    g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
    g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  out[blockIdx.x * 512 + tid] = sink;
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? atoi(argv[1]) : 1366;
  const size_t wbytes = (size_t)CONVS * 40 * 16384;
  std::vector<unsigned short> hw(wbytes / 2);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0x2000 + (i * 7919 % 0x1000);
  uint4* w;
  float* out;
  (void)hipMalloc(&w, wbytes);
  (void)hipMalloc(&out, (size_t)grid * 512 * 4);
  (void)hipMemcpy(w, hw.data(), wbytes, hipMemcpyHostToDevice);
  const size_t lds = 140 * 1024;
  (void)hipFuncSetAttribute((const void*)&kbench<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  (void)hipFuncSetAttribute((const void*)&kbench<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto run = [&](const char* name, auto kern, int threads) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int i = 0; i < 20; ++i) kern<<<grid, threads, lds>>>(w, out, 7);
    (void)hipEventRecord(a);
    for (int i = 0; i < 50; ++i) kern<<<grid, threads, lds>>>(w, out, 7);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long clk[4];
    (void)hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk));
    printf("%-28s grid %d: %7.1f us/launch, clock %4.0f MHz, wg0 %6.0f cycles/conv (MFMA floor 27648)\n", name, grid,
           ms * 1000 / 50, (double)clk[0] / clk[1] * 100.0, (double)clk[0] / CONVS);
  };
  for (int round = 0; round < 2; ++round) {
    run("16x16x32", kbench<0, 0>, 512);
    run("16x16x32 pairs in step (product)", kbench<0, 128>, 512);
    run("pairs, taps unrolled by 3", kbench<0, 128, 4, 3>, 512);
    run("pairs, taps unrolled by 9", kbench<0, 128, 4, 9>, 512);
    run("pairs, PF2", kbench<0, 128 | 512>, 512);
    run("pairs, PF2, unrolled by 3", kbench<0, 128 | 512, 4, 3>, 512);
    run("M quarters x N halves", kbench<3, 0>, 512);
    run("M quarters x N halves no-B", kbench<3, 1>, 512);
    run("pairs in step no-B", kbench<0, 129>, 512);
    run("16x16x32 term-major (dbuf A)", kbench<0, 8>, 512);
    run("term-major ring (product regs)", kbench<0, 32>, 512);
    run("term-major ring pf2", kbench<0, 48>, 512);
    run("term-major ring lagged", kbench<0, 96>, 512);
    run("w4 term-major ring lagged", kbench<0, 96, 8>, 256);
    run("w4 (1 wave/SIMD, 8 blk)", kbench<0, 0, 8>, 256);
    run("w4 term-major (dbuf A)", kbench<0, 8, 8>, 256);
    run("w4 term-major ring", kbench<0, 32, 8>, 256);
    run("w4 term-major ring pf2", kbench<0, 48, 8>, 256);
  }
  return 0;
}
