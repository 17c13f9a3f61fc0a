// Standalone check + timing of conv16_kernel (csrc/az_conv16.hip) on random
// data: split16 input rows, random 3x3 (+1x1 residual) weights, compared with
// a float64 direct convolution of the UNSPLIT fp32 input on sampled boards.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 profiles/micro/conv16_bench.cpp -o conv16_bench
//   ./conv16_bench boards H W mb mode(0 conv, 1 conv+res, 2 conv+res+heads) iters
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../custom-alphazero_amd/csrc/az_conv16.hip"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

static void split_host(const float* x, uint16_t* row) {  // one pixel: 128 channels
  for (int c = 0; c < 128; ++c) {
    const _Float16 h = (_Float16)x[c];
    const _Float16 l = (_Float16)((x[c] - (float)h) * 4096.f);
    memcpy(row + c, &h, 2);
    memcpy(row + 128 + c, &l, 2);
  }
}
static float unsplit(const uint16_t* row, int c) {
  _Float16 h, l;
  memcpy(&h, row + c, 2);
  memcpy(&l, row + 128 + c, 2);
  return (float)h + (float)l * (1.f / 4096.f);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 870;
  const int H = argc > 2 ? atoi(argv[2]) : 6, W = argc > 3 ? atoi(argv[3]) : 7;
  const int wm = argc > 4 ? atoi(argv[4]) : 4;  // M blocks per tile
  const int mode = argc > 5 ? atoi(argv[5]) : 1;
  const int iters = argc > 6 ? atoi(argv[6]) : 50;
  const int HW = H * W, F = 128, rows = B * HW;
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U01(0.f, 1.f), Upm(-1.f, 1.f);
  std::vector<float> x((size_t)rows * F), xr((size_t)rows * F);
  for (auto& v : x) v = U01(rng) < 0.5f ? 0.f : 2.f * U01(rng);  // ReLU-like activations
  for (auto& v : xr) v = U01(rng) < 0.5f ? 0.f : 2.f * U01(rng);
  const double lim = std::sqrt(6.0 / (9 * F * 2));
  std::vector<double> w3((size_t)9 * F * F), wr((size_t)F * F);
  for (auto& v : w3) v = lim * Upm(rng);
  for (auto& v : wr) v = 2 * lim * Upm(rng);
  std::vector<float> bias(F);
  for (auto& v : bias) v = 0.1f * Upm(rng);
  std::vector<float> hw(3 * F + 3);
  for (auto& v : hw) v = 0.1f * Upm(rng);
  const bool res = mode >= 1, heads = mode == 2;

  std::vector<uint16_t> xs((size_t)rows * 256), xrs((size_t)rows * 256);
  for (int r = 0; r < rows; ++r) {
    split_host(&x[(size_t)r * F], &xs[(size_t)r * 256]);
    split_host(&xr[(size_t)r * F], &xrs[(size_t)r * 256]);
  }
  const int e = az::conv16_prescale(w3.data(), w3.size(), res ? wr.data() : nullptr, res ? wr.size() : 0);
  std::vector<uint16_t> pack;
  az::conv16_pack(w3.data(), F, res ? wr.data() : nullptr, e, pack);

  void *d_in, *d_res, *d_w, *d_out, *d_bias, *d_hw, *d_feat;
  unsigned long long* d_err;
  CK(hipMalloc(&d_in, xs.size() * 2));
  CK(hipMalloc(&d_res, xrs.size() * 2));
  CK(hipMalloc(&d_w, pack.size() * 2));
  CK(hipMalloc(&d_out, (size_t)rows * 512));
  CK(hipMalloc(&d_bias, F * 4));
  CK(hipMalloc(&d_hw, hw.size() * 4));
  CK(hipMalloc(&d_feat, (size_t)rows * 16));
  CK(hipMalloc(&d_err, 8));
  CK(hipMemcpy(d_in, xs.data(), xs.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_res, xrs.data(), xrs.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_w, pack.data(), pack.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_bias, bias.data(), F * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_hw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(d_err, 0, 8));

  az::Conv16Args a;
  a.in = d_in;
  a.res_in = res ? d_res : nullptr;
  a.wpack = d_w;
  a.bias = (const float*)d_bias;
  a.oscale = std::ldexp(1.f, e - 12);
  a.out = d_out;
  if (heads) {
    const float* h = (const float*)d_hw;
    a.heads = az::Conv16Heads{h, h + 2 * F, h + 2 * F + 2, h + 3 * F + 2, (float4*)d_feat};
  }
  a.n_max = B;
  a.H = H;
  a.W = W;
  a.mb = wm;
  a.err = d_err;
  az::launch_conv16(a, 0);
  CK(hipDeviceSynchronize());

  // ---- check sampled boards against float64
  std::vector<uint16_t> out((size_t)rows * 256);
  std::vector<float> feat((size_t)rows * 4);
  CK(hipMemcpy(out.data(), d_out, out.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(feat.data(), d_feat, feat.size() * 4, hipMemcpyDeviceToHost));
  double max_err = 0, max_ref = 0;
  const int sample[3] = {0, B / 2, B - 1};
  for (int sb : sample) {
    for (int p = 0; p < HW; ++p) {
      const int y = p / W, xx = p % W, r = sb * HW + p;
      std::vector<double> acc(F, 0.0);
      for (int tap = 0; tap < 9; ++tap) {
        const int ny = y + tap / 3 - 1, nx = xx + tap % 3 - 1;
        if (ny < 0 || ny >= H || nx < 0 || nx >= W) continue;
        const float* xi = &x[((size_t)sb * HW + ny * W + nx) * F];
        for (int c = 0; c < F; ++c)
          if (xi[c] != 0.f)
            for (int o = 0; o < F; ++o) acc[o] += (double)xi[c] * w3[((size_t)tap * F + c) * F + o];
      }
      if (res)
        for (int c = 0; c < F; ++c) {
          const float v = xr[(size_t)r * F + c];
          if (v != 0.f)
            for (int o = 0; o < F; ++o) acc[o] += (double)v * wr[(size_t)c * F + o];
        }
      double s[3] = {0, 0, 0};
      for (int o = 0; o < F; ++o) {
        const double yv = std::max(acc[o] + bias[o], 0.0);
        if (heads) {
          s[0] += yv * hw[2 * o];
          s[1] += yv * hw[2 * o + 1];
          s[2] += yv * hw[2 * F + 2 + o];
        } else {
          const double got = unsplit(&out[(size_t)r * 256], o);
          max_err = std::max(max_err, std::fabs(got - yv));
          max_ref = std::max(max_ref, std::fabs(yv));
        }
      }
      if (heads) {
        const double ref[3] = {std::max(s[0] + hw[2 * F], 0.0), std::max(s[1] + hw[2 * F + 1], 0.0),
                               std::max(s[2] + hw[3 * F + 2], 0.0)};
        for (int k = 0; k < 3; ++k) {
          max_err = std::max(max_err, std::fabs(feat[(size_t)r * 4 + k] - ref[k]));
          max_ref = std::max(max_ref, std::fabs(ref[k]));
        }
      }
    }
  }
  unsigned long long err_flag = 0;
  CK(hipMemcpy(&err_flag, d_err, 8, hipMemcpyDeviceToHost));

  // ---- timing
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  for (int i = 0; i < 5; ++i) az::launch_conv16(a, 0);
  CK(hipEventRecord(t0, 0));
  for (int i = 0; i < iters; ++i) az::launch_conv16(a, 0);
  CK(hipEventRecord(t1, 0));
  CK(hipEventSynchronize(t1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, t0, t1));
  const double us = 1e3 * ms / iters;
#ifdef AZ_C16_STAMPS
  {  // phase clocks of the last launch per tile: prologue (slab DMA), K loop, epilogue; shader clock
    static unsigned long long st[8192][6];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(az::g_c16_stamps), sizeof(st)));
    double ph[3] = {0, 0, 0}, clk = 0, t0 = 1e300, t1 = 0;
    int n = 0;
    for (int w = 0; w < 8192; ++w) {
      if (!st[w][0] || st[w][3] < st[w][0] || st[w][5] <= st[w][4]) continue;
      ++n;
      for (int k = 0; k < 3; ++k) ph[k] += (double)(st[w][k + 1] - st[w][k]);
      clk += (double)(st[w][3] - st[w][0]) / (double)(st[w][5] - st[w][4]) * 0.1;  // GHz (realtime 100 MHz)
      t0 = std::min(t0, (double)st[w][4]);
      t1 = std::max(t1, (double)st[w][5]);
    }
    if (n)
      fprintf(stderr, "stamps: %d tiles, mean cycles prologue %.0f loop %.0f epilogue %.0f, clock %.2f GHz, "
              "first start to last end %.1f us\n", n, ph[0] / n, ph[1] / n, ph[2] / n, clk / n, (t1 - t0) / 100.0);
  }
#endif
  const int nks = res ? 40 : 36;
  const double issued = (double)rows * F * 32.0 * nks * 2 * 3;         // fp16 MFMA FLOP issued
  const double direct = (double)rows * F * F * 2 * (9 + (res ? 1 : 0));  // algorithmic
  printf("{\"boards\": %d, \"H\": %d, \"W\": %d, \"wm\": %d, \"mode\": %d, \"us\": %.2f, "
         "\"issued_tflops\": %.1f, \"frac_f16_peak\": %.4f, \"algorithmic_tflops\": %.1f, "
         "\"max_abs_err\": %.3e, \"max_ref\": %.3f, \"rel\": %.3e, \"prescale\": %d, \"overflow_flag\": %llu}\n",
         B, H, W, wm, mode, us, issued / us * 1e-6, issued / us * 1e-6 / 2500.0, direct / us * 1e-6, max_err,
         max_ref, max_err / std::max(max_ref, 1e-30), e, err_flag);
  return 0;
}
