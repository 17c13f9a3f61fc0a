// Microbenchmark: v_mfma_f32_32x32x2_f32 throughput with 1, 2 or 4
// independent accumulator chains per wave, 1 or 2 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_chain.hip -o mfma_chain
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void chain(float* out, int iters, float a0, float b0) {
  f32x16 acc[NACC];
  for (int k = 0; k < NACC; ++k)
    for (int i = 0; i < 16; ++i) acc[k][i] = 0.f;
  float a = a0 + threadIdx.x, b = b0 - threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16 / NACC; ++s)
#pragma unroll
      for (int k = 0; k < NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[k], 0, 0, 0);
  }
  float t = 0.f;
  for (int k = 0; k < NACC; ++k)
    for (int i = 0; i < 16; ++i) t += acc[k][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

template <int NACC>
void run(int blocks_per_cu, float* out) {
  const int cus = 256, iters = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  chain<NACC><<<cus * blocks_per_cu, 256>>>(out, 10, 1.f, 2.f);
  hipEventRecord(e0);
  chain<NACC><<<cus * blocks_per_cu, 256>>>(out, iters, 1.f, 2.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2.0 * 32 * 32 * 2 * 16.0 * iters * 4 * cus * blocks_per_cu;
  printf("acc=%d waves/SIMD=%d: %.1f TFLOP/s (%.1f%% of 157.3)\n", NACC, blocks_per_cu,
         flop / ms / 1e9, 100.0 * flop / ms / 1e9 / 157.3);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 4 * 256 * sizeof(float));
  for (int w = 1; w <= 2; ++w) {
    run<1>(w, out);
    run<2>(w, out);
    run<4>(w, out);
  }
  return 0;
}
