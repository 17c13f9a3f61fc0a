// Microbenchmark (diagnostic, not product code): cycles per
// v_mfma_f32_16x16x32_f16 in the tower K loop's issue pattern -- 4 M blocks
// x 2 N blocks x 3 products per k-step -- for one or two waves per SIMD, with
// each accumulator's 3 products back to back (chain) or interleaved, and
// with or without a few VALU fillers per k-step.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_rate profiles/mfma_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int ORDER, int FILL>
__global__ __launch_bounds__(512) void rate(const h8* __restrict__ in, float* __restrict__ out,
                                            unsigned long long* __restrict__ cyc, int steps) {
  extern __shared__ float pad[];  // 100 KB: one workgroup per CU
  if (steps < 0) pad[threadIdx.x] = 0.f;
  h8 a[4][2], b[4];
  for (int i = 0; i < 4; ++i) {
    a[i][0] = in[threadIdx.x % 64 + i];
    a[i][1] = in[threadIdx.x % 64 + i + 4];
    b[i] = in[threadIdx.x % 64 + 8 + i];
  }
  f4 c[4][2];
  for (int m = 0; m < 4; ++m)
    for (int n = 0; n < 2; ++n) c[m][n] = f4{0.f, 0.f, 0.f, 0.f};
  int x = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if (ORDER == 0) {
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[2 * n], a[m][1], c[m][n], 0, 0, 0);
          c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[2 * n + 1], a[m][0], c[m][n], 0, 0, 0);
          c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[2 * n], a[m][0], c[m][n], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[2 * n + (k == 1)], a[m][k == 0], c[m][n], 0, 0, 0);
      }
      if (FILL) {
#pragma unroll
        for (int f = 0; f < FILL; ++f) x = x * 3 + 1;
      }
    }
    asm volatile("" : "+v"(x));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  for (int m = 0; m < 4; ++m)
    for (int n = 0; n < 2; ++n) acc += c[m][n][0] + c[m][n][1] + c[m][n][2] + c[m][n][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc + x;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

template <int ORDER, int FILL>
void run(const char* name, int threads, h8* in, float* out, unsigned long long* cyc) {
  const int steps = 2000, blocks = 256;
  hipFuncSetAttribute(reinterpret_cast<const void*>(&rate<ORDER, FILL>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
  for (int rep = 0; rep < 2; ++rep) rate<ORDER, FILL><<<blocks, threads, 100 * 1024>>>(in, out, cyc, steps);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 8);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  double mx = 0, sum = 0;
  const int waves = threads / 64;
  for (int b = 0; b < blocks; ++b)
    for (int w = 0; w < waves; ++w) {
      mx = std::max(mx, (double)h[b * 8 + w]);
      sum += h[b * 8 + w];
    }
  const double mfma_per_simd = 24.0 * steps * (waves > 4 ? 2 : 1);
  printf("%-28s waves/SIMD %d: s_memtime per MFMA per SIMD (max wave) %.2f, mean wave %.2f\n", name,
         waves > 4 ? 2 : 1, mx / mfma_per_simd, sum / (blocks * waves) / mfma_per_simd);
}

int main() {
  h8* in;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&in, 256 * sizeof(h8));
  hipMemset(in, 0, 256 * sizeof(h8));
  hipMalloc(&out, 256 * 512 * sizeof(float));
  hipMalloc(&cyc, 256 * 8 * 8);
  run<0, 0>("chain", 256, in, out, cyc);
  run<0, 0>("chain", 512, in, out, cyc);
  run<1, 0>("interleaved", 256, in, out, cyc);
  run<1, 0>("interleaved", 512, in, out, cyc);
  run<0, 2>("chain + 2 VALU per block", 256, in, out, cyc);
  run<0, 2>("chain + 2 VALU per block", 512, in, out, cyc);
  run<0, 6>("chain + 6 VALU per block", 256, in, out, cyc);
  run<0, 6>("chain + 6 VALU per block", 512, in, out, cyc);
  return 0;
}
