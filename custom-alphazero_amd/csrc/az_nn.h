// az_nn.h -- device-side network weights and the forward launchers.
#pragma once
#include <vector>

#include "../../include/az.h"
#include "az_device.h"

namespace az {

// Folded (BatchNorm-in) fp32 weights resident in HBM.  Layouts are chosen for
// the kernels, not copied from Keras: conv weights are [Cout][K] with K
// contiguous (K = tap*Cin + c), so a 32-wide K chunk of 128 output channels is
// a [128][32] tile loaded with 16-byte reads.
struct NetDev {
  int filters = 128, depth = 0, hidden = 256;
  int algo = 0;  // AZ_CONV_WINOGRAD / AZ_CONV_DIRECT
  int wino_ksplit = 1;  // 32-tile Winograd kernel: 1, or 2 = two chunk groups per workgroup
  int wino_tiles = 32;  // tiles per workgroup: 32 (wino_conv_kernel) or 16 (wino16_conv_kernel);
                        // one variant for every conv of a network (set before load_network)
  int wino_x3 = 0;      // 16 tiles: 1 = wino16x_conv_kernel (fp32 products from three bf16 terms)
  int in_ch = 4;            // input planes: 4 (Connect-N) or 118 (chess, padded to F)
  float* stem_w = nullptr;  // [36][F]  (k = tap*4 + c), in_ch == 4
  float* stem_u = nullptr;  // Winograd U of the zero-padded stem [3][3][F][F], in_ch > 4
  float* stem_b = nullptr;  // [F]
  std::vector<float*> c1_w, c1_b;  // fragment-packed [9F x F], [F]
  std::vector<float*> c2_w, c2_b;  // fragment-packed [10F x F] (conv2 taps, then 1x1 residual), [F]
  std::vector<float*> u1_w, u2_w;  // Winograd U[16][F][F], packed (az_engine.hip pack_wino)
  std::vector<float*> r2_w;        // 1x1 projection residual [F][F], Winograd fragment order
  float *pc_w = nullptr, *pc_b = nullptr;  // policy conv [F][2], [2]
  float *vc_w = nullptr, *vc_b = nullptr;  // value conv [F], [1]
  float *pd_w = nullptr, *pd_b = nullptr;  // policy dense [2HW][A], [A]
  float* pd_wt = nullptr;  // A > kMaxActions (chess): [ceil(A/64)][2HW][64], one contiguous slab per
                           // policy_dense_kernel column tile, zero past A
  float *v1_w = nullptr, *v1_b = nullptr;  // value dense1 [HW][hidden], [hidden]
  float *v2_w = nullptr, *v2_b = nullptr;  // value dense2 [hidden], [1]
  bool ready = false;
};

// hipEvent pairs around the conv launches of every forward while enabled, so
// bench.py can price the dominant kernel live (roofline.achieved).  `ref` is
// an event the engine records when timing starts: intervals of all lanes are
// placed on one device clock, so their union (time in which any conv ran)
// can be taken next to the summed durations.
struct ConvTimer {
  bool enabled = false;
  hipEvent_t* ref = nullptr;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  double total_ms = 0.0;
  long long launches = 0;
  std::vector<std::pair<double, double>> intervals;  // [start, end) ms after *ref
  void begin(hipStream_t s) {
    if (!enabled) return;
    if (used + 2 > pool.size()) {
      for (int i = 0; i < 256; ++i) {
        hipEvent_t e;
        // timing only: no system-scope fence (a default event's cache
        // writeback/invalidate cost ~12 us between the kernels it sits between)
        (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
        pool.push_back(e);
      }
    }
    (void)hipEventRecord(pool[used++], s);
  }
  void end(hipStream_t s, int n_launches) {
    if (!enabled) return;
    (void)hipEventRecord(pool[used++], s);
    launches += n_launches;
  }
  // call after a stream synchronize: folds recorded pairs into total_ms
  void flush() {
    for (size_t i = 0; i + 1 < used; i += 2) {
      float ms = 0.f, a = 0.f, b = 0.f;
      (void)hipEventElapsedTime(&ms, pool[i], pool[i + 1]);
      total_ms += ms;
      if (ref && hipEventElapsedTime(&a, *ref, pool[i]) == hipSuccess &&
          hipEventElapsedTime(&b, *ref, pool[i + 1]) == hipSuccess)
        intervals.emplace_back(a, b);
    }
    used = 0;
  }
  void reset() {
    used = 0;
    total_ms = 0.0;
    launches = 0;
    intervals.clear();
  }
  ~ConvTimer() {
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

void launch_encode(const Board* boards, const int* count, int n_max, int HW, float* x,
                   hipStream_t s);
void launch_legal_mask(const Board* boards, int n, const GameCfg& g, uint8_t* mask,
                       hipStream_t s);
// Winograd conv: input channels per LDS chunk (16 or 32; the host packing
// follows it) and the packing index of a weight in the kernel's B stream
#ifndef AZ_WINO_CK
#define AZ_WINO_CK 32
#endif
constexpr int kWinoCK = AZ_WINO_CK;
size_t wino_pack_index(int xi, int cin, int cout);
size_t wino16_pack_index(int xi, int cin, int cout);  // az_wino16.hip
size_t wino16x_pack_index(int xi, int cin, int cout, int k);  // az_wino16x.hip (bf16 units)
size_t wino16x_res_index(int cin, int cout, int k);
// 16-tile variant on v_mfma_f32_16x16x4_f32 (small launches; az_wino16.hip)
struct HeadConv;
void launch_wino16_conv(const float* in, const float* res_in, const float* upack, const float* rpack,
                        const float* bias, float* out, const int* count, int n_max, int H, int W,
                        hipStream_t s, const HeadConv* heads = nullptr, int first_chunk = 0);
void launch_wino16x_conv(const float* in, const float* res_in, const float* upack, const float* rpack,
                         const float* bias, float* out, const int* count, int n_max, int H, int W,
                         hipStream_t s, const HeadConv* heads = nullptr, int first_chunk = 0);
// The heads' 1x1 convolutions (policy F->2, value F->1, each + folded BN +
// ReLU, model.py:68-149), fused into the last block's conv2 epilogue: feat =
// [boards][HW] float4 (policy ch 0, policy ch 1, value, 0); the block output
// itself is then never written.
struct HeadConv {
  const float* wpc;  // [F][2]
  const float* bpc;  // [2]
  const float* wvc;  // [F]
  const float* bvc;  // [1]
  float4* feat;      // null: write the block output instead
};
// ksplit = 2: the two-chunk-group variant (small batches; az_wino.hip)
void launch_wino_conv(const float* in, const float* res_in, const float* upack,
                      const float* rpack, const float* bias, float* out, const int* count,
                      int n_max, int H, int W, hipStream_t s, const HeadConv* heads = nullptr,
                      int ksplit = 1);
// x: [n][HW][4]; count (device int, may be null -> n_max) is the live batch.
// boards (optional): one-hot input straight from the eval queue's boards
// (bitwise the same outputs as encoding them into x first)
// Folds and uploads the network weights (Keras names, model/weights.py);
// device buffers are appended to `owned` (az_engine.hip)
int load_network(NetDev& net, const ::az_tensor* tensors, int n, int in_ch, int HW, int A,
                 double eps, std::vector<void*>& owned);
// x: [n][HW][4] (in_ch == 4) or [n][HW][F] zero-padded planes (in_ch > 4)
void launch_forward(const NetDev& net, const float* x, const int* count, int n_max, int H, int W,
                    int A, float* act_a, float* act_b, float* act_c, float* probs, float* values,
                    hipStream_t s, ConvTimer* timer, const Board* boards = nullptr,
                    int stem_first_chunk = 0);

}  // namespace az
