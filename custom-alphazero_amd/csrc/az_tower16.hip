// az_tower16.hip -- the whole Connect-N policy/value forward in ONE kernel
// (model/tensorflow/model.py:152-188 at inference): stem, the residual
// tower's 2*depth 3x3 convs, the heads' 1x1 convs, the dense layers, softmax
// and tanh.
//
// A workgroup owns WHOLE boards (Connect-4: 3 boards = 126 pixel rows of a
// 128-row tile) and keeps their activations in LDS from the stem to the
// heads.  A 3x3 'same' conv never reads outside its own board (off-board
// neighbours are the zero row), so a tile needs no halo, no layer's output
// makes an HBM round trip and a forward is one launch instead of eleven.
// Per-layer work is the split16 scheme of az_conv16.hip: activations
// x ~= t0 + t1 (fp16 terms, t1 unscaled here) and prescaled weights
// w' = b0 + b1 * 2^-12 as fp16 term pairs, three v_mfma_f32_16x16x32_f16 per
// k-step into one fp32 accumulator (t1*B0 + t0*b1 + t0*B0, B0 = 2^12 b0), so
// every layer is fp32-accurate (network error vs float64 ~1e-7).
//
// Workgroup = 8 waves (two per SIMD): wave w takes M half w & 1 (MBW 16-row
// blocks) and N quarter w >> 1 (32 output channels) -- in general M part
// w % NWM, N quarter w / NWM (variants/nwm4.py: NWM = 4, 16 waves).  The two waves loading
// one N quarter's weight fragments are then w and w ^ 1: a workgroup's waves
// go to the SIMDs in the order 0, 2, 1, 3, so they sit on different SIMDs
// and are both the older (waves 0-3) or both the younger (4-7) wave of their
// SIMD -- they run in step and the second request for a fragment finds it in
// the CU's L1 (round 4: 975 vs 1008 us per 4096-board forward, +3.2%
// games/s, profiles/r4/shape_runs/ab_pairl1.txt; with M half w >> 2 the pair
// shared a SIMD, the younger ran ~6 k-steps behind and missed L1).  The weights are the
// MFMA's A operand, so a lane's accumulators are 4 consecutive channels of
// one pixel: an epilogue writes its split16 terms to LDS as 8-byte stores
// straight from the registers.  B fragments (host-packed, conv16_pack) stream
// from L2 into registers PF k-steps ahead by buffer loads; activation
// fragments are read from LDS one k-step ahead, each block's after the next
// block's MFMAs (34-slot rows keep every ds_read_b128 lane group on 16
// distinct bank quads for any tap shift).
//
// Slot plan (tower16_slot_plan): the tile's slots are ordered so that whole
// 16-row blocks hold pixels of one board edge; such a border block skips the
// three taps past its edge (their MFMAs would add exact zeros).  The
// activation image stays in natural row order; a slot's pixel word names its
// row.
//
// The block's 1x1 projection residual (base_layers.py:95-125) is computed in
// conv1's phase (4 k-steps on the block input's own rows, into a second
// accumulator), because conv1's output then overwrites the block input in
// LDS; conv2 accumulates its taps on top of it.
//
// Range: a split16 term is fp16, so a stored activation must stay within
// +-32752.  Each board carries a power-of-two scale per activation buffer:
// a layer output whose board maximum exceeds the range is stored as
// y * 2^-s (s the smallest that fits) and the next conv multiplies its
// accumulator back by 2^s (exact).  The scale depends only on the board's
// own values, so results stay batch invariant; with no overflow (every
// network we have seen) s = 0 everywhere and nothing is rescaled.
//
// Every output element is summed in a fixed order (k-step, then term; heads
// in a fixed tree), so a board's outputs do not depend on its position in
// the tile or on the rest of the batch -- the oracle replay tests rely on it.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <type_traits>

#include "az_nn.h"
#include "az_tree.h"
#include "az_kloop_asm.h"
#include "az_chess.h"

namespace az {

typedef _Float16 t_h8 __attribute__((ext_vector_type(8)));
typedef float t_f4 __attribute__((ext_vector_type(4)));

namespace {

constexpr float kRange = 32752.f;  // largest |x| a split16 term pair holds
// LDS activation rows: 34 16-byte slots (term 0 of the 128 channels in slots
// 0..15, term 1 in 16..31, two pad slots).  A row's slot s sits in bank quad
// (2 row + s) mod 16: a ds_read_b128 lane group (8 consecutive rows at slot g
// and the same 8 at g + 1) covers the even quads with one half and the odd
// ones with the other, for any tap shift, with no swizzle, and a chunk's slot
// is an immediate offset (PMC: a 33-slot pitch conflicted 2-way).  8 zero rows
// follow the tile: an off-board tap of row r reads zero row (r & 7), the quad
// its own row has.
constexpr int kPitch = 544;
constexpr int kZeroRows = 8;
// A tile slot's pixel word: (board << 16) | (y << 8) | x.  An empty slot (past
// the tile's boards, or a pad of the slot plan) has y = 127, off every board,
// so each of its taps reads a zero row; its x holds the LDS bank residue its
// zero-row reads take.  A slot's LDS row is its pixel's natural row
// board * HW + y * W + x (the activation image is in natural order whatever
// order the slots compute in); an empty slot's "row" is its residue.
__device__ __forceinline__ bool pix_ok(int yx) { return ((yx >> 8) & 255) != 127; }
__device__ __forceinline__ int pix_row(int yx, int HW, int W) {
  return pix_ok(yx) ? (yx >> 16) * HW + ((yx >> 8) & 255) * W + (yx & 255) : (yx & 7);
}

#ifdef AZ_T16_STAMPS  // diagnostic build only: phase clocks of wave 0 per workgroup (az_t16_stamps)
constexpr int kStampBlocks = 4096, kStamps = 64;
__device__ unsigned long long g_t16_stamps[kStampBlocks][kStamps];
#define T16_STAMP(k)                                                             \
  if (threadIdx.x == 0 && blockIdx.x < kStampBlocks) {                           \
    g_t16_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime();                  \
  }
#define T16_RSTAMP(k)                                                            \
  if (threadIdx.x == 0 && blockIdx.x < kStampBlocks) {                           \
    g_t16_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();              \
  }
// per wave of block 1: [c1 start, c1 end, c2 start, c2 end, HW_ID]
__device__ unsigned long long g_t16_wstamps[kStampBlocks][8][5];
#define T16_WSTAMP(d, k)                                                          \
  if ((d) == 1 && (threadIdx.x & 63) == 0 && blockIdx.x < kStampBlocks) {        \
    g_t16_wstamps[blockIdx.x][threadIdx.x >> 6][k] = __builtin_amdgcn_s_memtime(); \
    if ((k) == 0)                                                                 \
      g_t16_wstamps[blockIdx.x][threadIdx.x >> 6][4] =                            \
          (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                    \
  }
#define T16_STAMP4(k)  /* wave 4 (wave 0's SIMD partner) */                    \
  if (threadIdx.x == 256 && blockIdx.x < kStampBlocks) {                         \
    g_t16_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime();                  \
  }
#else
#define T16_STAMP4(k)
#define T16_WSTAMP(d, k)
#define T16_STAMP(k)
#define T16_RSTAMP(k)
#endif

// Pointers read from the TowerNet struct are generic to the compiler, and a
// generic load is a FLAT load: counted in both vmcnt and lgkmcnt and waited
// for with vmcnt(0) -- which waited out the whole B prefetch every k-step.
// Every global read goes through this cast (global_load_*).
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gbl(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}
// the same for class types (float4, uint4, Board): a global load of their bits
template <typename T>
__device__ __forceinline__ T gld(const T* p) {
  static_assert(sizeof(T) % 4 == 0, "32-bit words");
  typedef unsigned int V __attribute__((ext_vector_type(sizeof(T) / 4)));
  return __builtin_bit_cast(T, *(const __attribute__((address_space(1))) V*)p);
}


// The tower's activation terms: x ~= t0 + t1 with t0 = fp16_rn(x) and t1 =
// fp16_rn(x - t0) (the subtraction exact), NOT scaled by 2^12 like az_nn.h's
// split16: then t1 * B0 (B0 = 2^12 b0, the pack's main weight term) is the
// correction product at the main term's scale and the K loop needs no b0.
// t1 reaches the fp16 subnormals below |x| ~ 2^-3; its absolute error there
// is <= 2^-25, far inside the 1e-5 network tolerance (measured ~2e-8).
__device__ __forceinline__ void split_u4(const float4 v, uint2& t0, uint2& t1) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t p[2], q[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    p[i] = pk_f16(x[2 * i], x[2 * i + 1]);
    const az_h2 h = __builtin_bit_cast(az_h2, p[i]);
    q[i] = pk_f16(x[2 * i] - (float)h[0], x[2 * i + 1] - (float)h[1]);
  }
  t0 = make_uint2(p[0], p[1]);
  t1 = make_uint2(q[0], q[1]);
}
__device__ __forceinline__ void split_u8(const float (&x)[8], uint4& t0, uint4& t1) {
  uint2 a0, a1, b0, b1;
  split_u4(make_float4(x[0], x[1], x[2], x[3]), a0, a1);
  split_u4(make_float4(x[4], x[5], x[6], x[7]), b0, b1);
  t0 = make_uint4(a0.x, a0.y, b0.x, b0.y);
  t1 = make_uint4(a1.x, a1.y, b1.x, b1.y);
}

// wave64 reductions without LDS round trips: DPP inside each 16-lane row
// (xor 1, xor 2 by quad_perm, then rotations by 4 and 8), the four row
// totals combined by readlane; a fixed order, the result wave-uniform
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <typename F>
__device__ __forceinline__ float wreduce(float v, F op) {
  v = op(v, dpp_f<0xB1>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_f<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_f<0x124>(v));  // row_ror:4
  v = op(v, dpp_f<0x128>(v));  // row_ror:8
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return op(op(r0, r1), op(r2, r3));
}
__device__ __forceinline__ float wsum(float v) {
  return wreduce(v, [](float a, float b) { return a + b; });
}
__device__ __forceinline__ float wmax(float v) {
  return wreduce(v, [](float a, float b) { return fmaxf(a, b); });
}

// smallest s >= 0 with m * 2^-s <= kRange (m >= 0, finite)
__device__ __forceinline__ int range_exp(float m) {
  int s = 0;
  while (ldexpf(m, -s) > kRange) ++s;
  return s;
}

// Shared bookkeeping after the activation rows.
struct TowerSmem {
  int flag[2];              // overflow seen in the layer being stored (alternating by layer)
  int sc[2][kTowerMaxBoards];  // per-board scale exponent of the two activation buffers' contents
  unsigned bmax[kTowerMaxBoards];  // board maxima (float bits, values >= 0) on the rare rescale path
};

// store 4 channels (channel quad cq) of activation row r as split16 terms
__device__ __forceinline__ void put4(uint4* act, int r, int cq, const float4 y) {
  uint2 t0, t1;
  split_u4(y, t0, t1);
  char* q = reinterpret_cast<char*>(act) + r * kPitch + cq * 8;
  *reinterpret_cast<uint2*>(q) = t0;
  *reinterpret_cast<uint2*>(q + 256) = t1;
}

__device__ __forceinline__ float max4(const float4 v) { return fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)); }
__device__ __forceinline__ float4 scale4(const float4 v, float s) {
  return make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
}

// Store one layer's output (2*MBW float4 items per thread, values >= 0).  Optimistic at scale 0; if any
// value left the split16 range, the boards concerned are stored again at
// their scale.  Returns whether any board of this buffer is scaled (then
// sc_out holds the exponents).  Contains the barrier that publishes the
// stores.  `par` alternates per layer (flag[par] is this layer's).
template <int MBW>
__device__ __forceinline__ bool store_layer(uint4* act, int HW, int W, const int (&yx_)[MBW], int cq0, const float4 (&y)[2 * MBW],
                                            TowerSmem& sm, int par, int* sc_out, int nbrd,
                                            unsigned long long* err) {
  // item mb*2 + nb: the slot's LDS row (if it holds a pixel), channel quad
  // cq0 + 4 nb, board yx >> 16; rows and boards laundered (as in k_loop): the
  // addresses derived from them are recomputed here, not hoisted out of the
  // depth loop and spilled
  int row[MBW], brd[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    row[mb] = pix_ok(yx_[mb]) ? pix_row(yx_[mb], HW, W) : -1;
    brd[mb] = yx_[mb] >> 16;
    asm volatile("" : "+v"(row[mb]), "+v"(brd[mb]));
  }
  float vmax = 0.f;
#pragma unroll
  for (int i = 0; i < 2 * MBW; ++i)
    if (row[i / 2] >= 0) {
      vmax = fmaxf(vmax, max4(y[i]));
      put4(act, row[i / 2], cq0 + 4 * (i & 1), y[i]);
    }
  if (!(vmax <= kRange)) sm.flag[par] = 1;  // also NaN
  if (threadIdx.x == 0) sm.flag[par ^ 1] = 0;  // next layer's flag (nobody reads it before then)
  __syncthreads();
  if (!sm.flag[par]) return false;  // workgroup-uniform
  // rare: board maxima, then the scaled boards' rows again
  if ((int)threadIdx.x < nbrd) sm.bmax[threadIdx.x] = 0u;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2 * MBW; ++i)
    if (row[i / 2] >= 0) atomicMax(&sm.bmax[brd[i / 2]], __float_as_uint(max4(y[i])));
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2 * MBW; ++i) {
    if (row[i / 2] < 0) continue;
    const float m = __uint_as_float(sm.bmax[brd[i / 2]]);
    if (!(m <= 3.0e38f)) continue;  // inf/NaN: flagged below, nothing to rescale
    const int s = range_exp(m);
    if (s) put4(act, row[i / 2], cq0 + 4 * (i & 1), scale4(y[i], ldexpf(1.f, -s)));
  }
  if ((int)threadIdx.x < nbrd) {
    const float m = __uint_as_float(sm.bmax[threadIdx.x]);
    if (!(m <= 3.0e38f)) {
      if (err) atomicOr(err, kErrActRange);
      sc_out[threadIdx.x] = 0;
    } else {
      sc_out[threadIdx.x] = range_exp(m);
    }
  }
  __syncthreads();
  return true;
}

// One conv phase's K loop: R residual k-steps (the block input's own rows x
// the 1x1 projection weights, k-steps 36.. of the conv2 pack, into accr),
// then 9 taps x 4 channel chunks of 32 (into acc).  The taps are a runtime
// loop with the chunks unrolled inside: fully unrolled, the two phases made
// a 110 KB kernel (the instruction cache holds 64 KB).  Ring slots are the
// k-step mod 4 (R is 0 or 4), so every register index stays static.
template <int V>
using IC = std::integral_constant<int, V>;

// res_shift: the residual k-steps read the own rows res_shift rows from
// `act` (conv2 of the double-buffered tower reads X's rows beside H's taps);
// mid() runs between the residual k-steps and the taps.
struct NoMid {
  __device__ void operator()() const {}
};
// C0: input channel chunks below it are known zero and skipped (each tap
// runs chunks C0..3; the chess stem in self-play, planes 0-63)
template <int MBW, int R, int C0 = 0, typename Mid = NoMid>
__device__ __forceinline__ void k_loop(const uint4* __restrict__ act, const uint4* __restrict__ wmain,
                                       const uint4* __restrict__ wres, t_f4 (&acc)[MBW][2],
                                       t_f4 (&accr)[MBW][2], const int (&yx_)[MBW], int H, int W,
                                       int zrow, int nq, int lane, int skw, int res_shift = 0,
                                       Mid mid = Mid{}) {
  static_assert(R == 0 || R == 4, "ring slots = k-step mod NB, NB divides 4");
  static_assert(C0 == 0 || (R == 0 && C0 == 2), "skipped chunks: the stem only, an even count");
  // SIMD-pair priority by phase: each SIMD runs one of waves 0-3 (older)
  // and one of 4-7 (younger); the older wins the MFMA pipe by default and
  // finishes ~8k cycles ahead, after which its partner runs alone.  The
  // younger wave takes priority 1 for the residual steps and taps 0-5, the
  // older for taps 6-8, so both reach the barrier closer together (round 4:
  // 929-938 vs 964-970 us per 4096-board forward, +1.9% games/s,
  // profiles/r4/shape_runs/ab_prio2.txt).  The wave index goes through
  // readfirstlane so each s_setprio sits under a scalar branch (under a
  // per-lane branch both paths execute: round 3's per-k-step turn was a no-op)
  // B fragments one k-step ahead of their MFMAs (2 measured equal, 1 needs no spill)
  constexpr int PF = 1, NB = 2;
  const int gq = lane >> 4;
  // the tap geometry laundered through an empty asm per call: the k-loops sit
  // in the runtime depth loop, and without this the compiler hoists every
  // k-step's LDS address out of it (loop invariant) and spills them
  int r[MBW], yx[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    yx[mb] = yx_[mb];
    asm volatile("" : "+v"(yx[mb]));
    r[mb] = pix_row(yx[mb], H * W, W);
  }
  uint4 bq[NB][4];
  // k-step s of the phase (s < R: residual, k-steps 36.. of the conv2 pack)
  // -> its B fragments, by buffer loads: the pack's base in an SGPR
  // descriptor, the lane's offset in one VGPR, the k-step's in soffset, the 4
  // fragments as immediate offsets -- no 64-bit address arithmetic (and its
  // carry-hazard nop) per k-step
  const auto rs_m = __builtin_amdgcn_make_buffer_rsrc((void*)wmain, (short)0, 0x7fffffff, 0x00020000);
  const auto rs_r = __builtin_amdgcn_make_buffer_rsrc((void*)(R ? wres : wmain), (short)0, 0x7fffffff, 0x00020000);
  const int voff = ((nq * 2) * 2 * 64 + lane) * 16;
  auto load_bk = [&](int s, uint4(&dst)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const auto v = s < R ? __builtin_amdgcn_raw_buffer_load_b128(rs_r, voff + q * 1024, (36 + s) * 16384, 0)
                           : __builtin_amdgcn_raw_buffer_load_b128(rs_m, voff + q * 1024, (s - R) * 16384, 0);
      dst[q] = __builtin_bit_cast(uint4, v);
    }
  };

  // per M block: the byte address of the tap row's term-0 slot gq; chunk c
  // and term 1 are immediate offsets (+64 c, +256)
  int aaddr[MBW];
  const char* actb = reinterpret_cast<const char*>(act);
  // blocks [lo, hi) to the block input's own rows / to a runtime tap
  auto set_own = [&](int lo, int hi) {
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
      if (mb >= lo && mb < hi) aaddr[mb] = (pix_ok(yx[mb]) ? r[mb] + res_shift : zrow + (r[mb] & 7)) * kPitch + gq * 16;
  };
  auto set_tap = [&](int t, int lo, int hi) {
    const int dy = t / 3 - 1, dx = t - (t / 3) * 3 - 1;
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      if (mb < lo || mb >= hi) continue;
      const int py = (yx[mb] >> 8) & 255, px = yx[mb] & 255;
      const bool ok = py + dy >= 0 && py + dy < H && px + dx >= 0 && px + dx < W;
      const int sr = r[mb] + dy * W + dx;
      aaddr[mb] = (ok ? sr : zrow + (sr & 7)) * kPitch + gq * 16;
    }
  };
  // activation fragments in a ring of RING M blocks: after block mb's MFMAs
  // its slot takes block mb + RING -- of this k-step while that is < MBW, else
  // block mb + RING - MBW of the next one -- so RING - 1 blocks' MFMAs hide
  // each read (RING = MBW: every block's read is one k-step ahead).  At a tap
  // change a block's address moves after its last read of the old tap: blocks
  // < RING at the start of the tap's last k-step, blocks >= RING at the start
  // of the next tap's first.
  constexpr int RING = MBW > 4 ? 4 : MBW;
  // lagged reads (RING = MBW): a block's next fragments are read after the
  // NEXT block's MFMAs, not right after its own, so the ds_read never
  // overwrites registers an in-flight MFMA is still reading (the WAR hazard
  // the compiler pads with s_nop); the last block's read moves to the next
  // k-step, after its block 0.  With the buffer-load weight stream: +1.6%
  // games/s (profiles/r3/lag_buf_ab_bench.txt)
  constexpr bool LAG = RING == MBW && MBW > 1;
  uint4 aq[RING][2];
  auto load_a1 = [&](int chunk, int mb) {
    const char* q = actb + aaddr[mb] + 64 * chunk;
    aq[mb % RING][0] = *reinterpret_cast<const uint4*>(q);
    aq[mb % RING][1] = *reinterpret_cast<const uint4*>(q + 256);
  };
  // one k-step (chunk `chunk` of the current addresses): per M block its 6
  // MFMAs (t1*B0 + t0*b1 + t0*B0 per N block, smallest first), then the ring
  // read that follows it (next_chunk < 0: this is the loop's last k-step).
  // skc: blocks whose MFMAs this k-step skips (every row's tap is off its
  // board: they would add exact zeros); skn: blocks the next k-step skips (no
  // read for them; 0 across a tap change)
  auto kstep = [&](t_f4(&C)[MBW][2], const uint4(&b)[4], int chunk, int next_chunk, auto skc, auto skn,
                   bool first = false) {
    constexpr int SKC = decltype(skc)::value, SKN = decltype(skn)::value;
    const t_h8 B0[2] = {__builtin_bit_cast(t_h8, b[0]), __builtin_bit_cast(t_h8, b[2])};
    const t_h8 B1[2] = {__builtin_bit_cast(t_h8, b[1]), __builtin_bit_cast(t_h8, b[3])};
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      const t_h8 a0 = __builtin_bit_cast(t_h8, aq[mb % RING][0]), a1 = __builtin_bit_cast(t_h8, aq[mb % RING][1]);
      if (((SKC >> mb) & 1) == 0) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        C[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a1, C[mb][nb], 0, 0, 0);
        C[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B1[nb], a0, C[mb][nb], 0, 0, 0);
        C[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], a0, C[mb][nb], 0, 0, 0);
      }
      }
      if (LAG) {
        if (mb == 0) {
          if (!first && ((SKC >> (MBW - 1)) & 1) == 0) load_a1(chunk, MBW - 1);  // this k-step's, lagged
        } else if (next_chunk >= 0 && ((SKN >> (mb - 1)) & 1) == 0) {
          load_a1(next_chunk, mb - 1);
        }
      } else if (mb + RING < MBW) {
        if (((SKC >> (mb + RING)) & 1) == 0) load_a1(chunk, mb + RING);
      } else if (next_chunk >= 0 && ((SKN >> (mb + RING - MBW)) & 1) == 0) {
        load_a1(next_chunk, mb + RING - MBW);
      }
    }
    // the order above, kept: the weight loads of the k-step PF ahead first,
    // then per M block its six MFMAs and its two ring reads
    // (left alone, the scheduler bunched the reads and waited for all of
    // them, and for the weight loads just issued, in mid k-step)
    __builtin_amdgcn_sched_group_barrier(0x0020, 4, 0);  // VMEM reads
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      if (((SKC >> mb) & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x0008, 6, 0);  // MFMA
      const bool rd = LAG ? (mb == 0 ? !first && ((SKC >> (MBW - 1)) & 1) == 0
                                     : next_chunk >= 0 && ((SKN >> (mb - 1)) & 1) == 0)
                    : mb + RING < MBW ? ((SKC >> (mb + RING)) & 1) == 0
                                      : next_chunk >= 0 && ((SKN >> (mb + RING - MBW)) & 1) == 0;
      if (rd) __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);  // DS reads
    }
  };

#pragma unroll
  for (int k = 0; k < PF; ++k) load_bk(C0 + k, bq[(C0 + k) % NB]);
  if (R) set_own(0, MBW);
  else set_tap(0, 0, MBW);
#pragma unroll
  for (int mb = 0; mb < RING; ++mb) load_a1(C0, mb);
  const bool young = __builtin_amdgcn_readfirstlane((int)threadIdx.x) >= 256;
  auto prio = [&](bool hi) {
    if (hi) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };
  prio(young);
  // ---- residual k-steps (static)
#pragma unroll
  for (int s = 0; s < R; ++s) {
    __builtin_amdgcn_sched_barrier(0);
    load_bk(s + PF, bq[(s + PF) % NB]);
    // the next k-step is tap 0's first chunk: the ring's low blocks move now
    // (lagged: all but the last, whose read of this k-step is still to come)
    if (s + 1 == R) set_tap(0, 0, LAG ? MBW - 1 : RING);
    kstep(accr, bq[s % NB], s, s + 1 == R ? 0 : s + 1, IC<0>{}, IC<0>{}, s == 0);
  }
  if (R) mid();
  // ---- 9 taps x 4 chunks; per tap the blocks it skips (skw: 2 bits per tap,
  // blocks 0 and 1 of the wave, from the slot plan) select one of three bodies
  auto tap = [&](int t, auto skc) {
#pragma unroll
    for (int c = C0; c < 4; ++c) {
      __builtin_amdgcn_sched_barrier(0);
      // main k-step PF ahead (the prologue or the residual steps fetched the first PF)
      const int ahead = c + PF < 4 ? 4 * t + c + PF : 4 * (t + 1) + C0 + (c + PF - 4);
      if (c + PF < 4 || t < 8) load_bk(R + ahead, bq[(c + PF) % NB]);
      // the tap's high blocks (first k-step; tap 0 after the residual steps)
      if (c == C0 && RING < MBW && (t > 0 || R)) set_tap(t, RING, MBW);
      if (LAG && c == C0 && (t > 0 || R)) set_tap(t, MBW - 1, MBW);  // its lagged read comes after block 0
      const bool first = !R && t == 0 && c == C0;
      if (c < 3) {
        kstep(acc, bq[c % NB], c, c + 1, skc, skc, first);
      } else if (t < 8) {
        set_tap(t + 1, 0, LAG ? MBW - 1 : RING);
        kstep(acc, bq[c % NB], c, C0, skc, IC<0>{}, first);
      } else {
        kstep(acc, bq[c % NB], c, -1, skc, IC<0>{}, first);
      }
    }
  };
#pragma unroll 1
  for (int t = 0; t < 9; ++t) {
    // wave-uniform; never 3 (one edge per tap and half).  The dispatch's
    // shape moves the register allocation: this form spills 7 VGPRs outside
    // the loops, testing m == 2 first spilled 140 inside them (and ran the
    // kernel at half speed) -- tests/test_kernel_resources_cpu.py guards it
    const int m = (skw >> (2 * t)) & 3;
    if (t == 6) prio(!young);
    if (m == 0) tap(t, IC<0>{});
    else if (m == 1) tap(t, IC<1>{});
    else tap(t, IC<2>{});
  }
  __builtin_amdgcn_s_setprio(0);
}

#ifndef AZ_KLOOP_TERM  // 1: term-major k-steps (gen_kloop_asm.term_group_asm); 0: block-major
#define AZ_KLOOP_TERM 1  // (within 1% of each other and of the compiled loop: profiles/r5/ab_term.txt)
#endif
#ifndef AZ_KLOOP_PF  // 2: +1% games/s over 1 at configs[1] (profiles/r5/ab_kloop.txt)
#define AZ_KLOOP_PF 2
#endif
// k_loop with the groups of 4 k-steps in hand-scheduled assembly
// (az_kloop_asm.h, gen_kloop_asm.py; term-major by default): every
// accumulator sums the same products in the same order as k_loop's, so
// the same bits.  accm / accr: the accumulators of the taps / the residual
// steps (may be the same array).  The schedule is checked symbolically by
// tests/test_kloop_schedule_cpu.py and against the compiled ISA by
// tests/test_kernel_resources_cpu.py
template <int MBW, int R, int C0, typename Mid = NoMid>
__device__ __forceinline__ void k_loop_asm(const uint4* __restrict__ act, const uint4* __restrict__ wmain,
                                           const uint4* __restrict__ wres, t_f4 (&accm)[MBW][2],
                                           t_f4 (&accr)[MBW][2], const int (&yx_)[MBW], int H, int W,
                                           int zrow, int nq, int lane, int skw, int res_shift = 0,
                                           Mid mid = Mid{}) {
  static_assert(R == 0 || R == 4, "residual steps: none or the 1x1 projection's 4");
  static_assert(C0 == 0 || (R == 0 && C0 == 2), "skipped chunks: the stem only, an even count");
  const int gq = lane >> 4;
  int r[MBW], yx[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    yx[mb] = yx_[mb];
    asm volatile("" : "+v"(yx[mb]));
    r[mb] = pix_row(yx[mb], H * W, W);
  }
  // the weight streams' buffer descriptors as SGPR quads
  auto quad = [](const void* p) {
    const unsigned long long a = reinterpret_cast<unsigned long long>(p);
    return az_rsrc{(int)(unsigned)a, (int)(unsigned)(a >> 32) & 0xffff, 0x7fffffff, 0x00020000};
  };
  const az_rsrc rs_m = quad(wmain), rs_r = quad(R ? wres : wmain);
  const int voff = ((nq * 2) * 2 * 64 + lane) * 16;
  // LDS byte addresses (ds_read's operand): act's base + the row's offset
  const int lbase = (int)(size_t)((__attribute__((address_space(3))) const char*)(const char*)act) + gq * 16;
  auto own = [&](int(&a)[MBW]) {
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) a[mb] = (pix_ok(yx[mb]) ? r[mb] + res_shift : zrow + (r[mb] & 7)) * kPitch + lbase;
  };
  auto tap_addr = [&](int t, int(&a)[MBW]) {
    const int dy = t / 3 - 1, dx = t - (t / 3) * 3 - 1;
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      const int py = (yx[mb] >> 8) & 255, px = yx[mb] & 255;
      const bool ok = py + dy >= 0 && py + dy < H && px + dx >= 0 && px + dx < W;
      const int sr = r[mb] + dy * W + dx;
      a[mb] = (ok ? sr : zrow + (sr & 7)) * kPitch + lbase;
    }
  };
  // weight prefetch depth: PF k-steps ahead in NB buffers (2 ahead needs 4,
  // so a 4-k-step group keeps each buffer's k-step fixed; the stem's
  // 2-k-step groups prefetch 1 ahead)
  // (the 192-row tile's 6-block waves: 1 -- 2 spills 69 VGPRs there.  3, in
  // 8 buffers picked by the tap's parity -- gen_kloop_asm.nbufs -- spilled
  // 627 VGPRs in chess's 2-block waves, one body per parity)
  constexpr int PF = C0 == 0 && MBW < 6 ? AZ_KLOOP_PF : 1, NB = PF == 1 ? 2 : 4;
  az_u4 aq[MBW][2], bq[NB][4];
  int cur[MBW], nxt[MBW];
  // prologue (asm too: a compiler load here would leave the compiler waiting
  // for it, vmcnt(0) lgkmcnt(0), before every group of the loop)
  if (R) own(cur);
  else tap_addr(0, cur);
  KPro<MBW, C0, PF, AZ_KLOOP_TERM>::run(aq, bq, cur, voff, R ? rs_r : rs_m, R ? 36 * 16384 : C0 * 16384);
  const bool young = __builtin_amdgcn_readfirstlane((int)threadIdx.x) >= 256;
  auto prio = [&](bool hi) {
    if (hi) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };
  prio(young);
  if constexpr (R) {
    tap_addr(0, nxt);
    KGroup<MBW, 0, 0, PF, AZ_KLOOP_TERM>::run(accr, aq, bq, cur, nxt, voff, rs_r, rs_m, 36 * 16384, 0);
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) cur[mb] = nxt[mb];
    mid();
  }
  // 9 taps, each in three bodies by the wave's skip mask (slot plan: never 3);
  // the last tap's prefetch re-reads its own first k-steps (drained; a peeled
  // last tap without them -- the generator's HASNEXT = 0 groups -- made the
  // allocator spill 400-550 VGPRs in the 128-row kernels)
  constexpr int O = AZ_KLOOP_TERM;
#pragma unroll 1
  for (int t = 0; t < 9; ++t) {
    if (t == 6) prio(!young);
    if (t < 8) tap_addr(t + 1, nxt);
    else {
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) nxt[mb] = cur[mb];
    }
    const int m = (skw >> (2 * t)) & 3;
    const int sc = 4 * t * 16384, sn = t < 8 ? (4 * (t + 1) + C0) * 16384 : sc + C0 * 16384;
    if (m == 0) KGroup<MBW, C0, 0, PF, O>::run(accm, aq, bq, cur, nxt, voff, rs_m, rs_m, sc, sn);
    else if (m == 1) KGroup<MBW, C0, (MBW > 1 ? 1 : 0), PF, O>::run(accm, aq, bq, cur, nxt, voff, rs_m, rs_m, sc, sn);
    else KGroup<MBW, C0, (MBW > 1 ? 2 : 0), PF, O>::run(accm, aq, bq, cur, nxt, voff, rs_m, rs_m, sc, sn);
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) cur[mb] = nxt[mb];
  }
  KDrain<MBW, NB>::run(accm, aq, bq);
  __builtin_amdgcn_s_setprio(0);
}

// the tower's K loop: the assembly groups; the compiled loop (k_loop) stays
// selectable for A/B runs of the two (EXTRA=-DAZ_KLOOP_CC: a diagnostic
// build, its build flags say so)
#ifdef AZ_KLOOP_CC
#define AZ_KLOOP k_loop
#else
#define AZ_KLOOP k_loop_asm
#endif

// LDS-DMA of n_u4 16-byte words from global src into LDS dst (both
// 16-byte aligned), the workgroup's waves in turn: no VGPRs, completes in the
// background (the first vmcnt wait of a K loop covers it)
template <int NT>
__device__ __forceinline__ void dma_to_lds(uint4* dst, const float* src, int n_u4, int wave, int lane) {
  if (n_u4 <= 0) return;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, n_u4 * 16, 0x00020000);
  for (int base = wave * 64; base < n_u4; base += NT) {  // wave-uniform
    const int i = base + lane;
    const unsigned voff = i < n_u4 ? (unsigned)(i * 16) : 0x80000000u;  // past the end: range-checked to 0
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(dst + base), 16,
                                             voff, 0, 0, 0);
  }
}

// MBT 16-row M blocks per tile (8: 128 rows, 6: 96); NWM wave groups over M
// (2 = 8 waves, two per SIMD, each MBT/2 blocks).  ROWS: the input-row form
// (chess, launch_tower16_rows): the stem is a 3x3 conv over F (padded) input
// channels read from split16 rows, and the kernel ends with the heads' 1x1
// convs (per pixel float4 features into feat) -- the dense heads (1880
// logits) run in their own kernels
template <int MBT, int NWM, bool ROWS, bool DB>
__device__ __forceinline__ void tower16_tile(const TowerNet* __restrict__ net, const Board* __restrict__ boards,
                                             const float4* __restrict__ x, const uint4* __restrict__ rows,
                                             int n, int H, int W, int A, int bpw, float* __restrict__ probs,
                                             float* __restrict__ values, float4* __restrict__ feat,
                                             int first_chunk, unsigned long long* __restrict__ err,
                                             TowerLeaves lv) {
  constexpr int MBW = MBT / NWM;  // M blocks per wave
  constexpr int TR = 16 * MBT;    // tile rows
  constexpr int NT = NWM * 256;
  extern __shared__ __attribute__((aligned(16))) uint4 act[];  // [TR + kZeroRows] rows of kPitch bytes
  const TowerNet& T = *net;
  // activation buffers X (block input) and H (conv1 output): two tiles around
  // the shared zero rows when the LDS holds them (T.dbuf: an epilogue writes
  // the other tile, so a wave that finishes its K loop stores its outputs
  // while its SIMD partner still computes, and one barrier per layer
  // publishes them), else one tile updated in place behind a second barrier
  constexpr bool dbuf = DB;
  uint4* const bufX = act;
  uint4* const bufH = dbuf ? act + (TR + kZeroRows) * (kPitch / 16) : act;
  const int zX = TR, zH = dbuf ? -kZeroRows : TR;  // each tile's zero rows, relative to it
  TowerSmem& sm = *reinterpret_cast<TowerSmem*>(reinterpret_cast<char*>(act) +
                                                ((dbuf ? 2 : 1) * TR + kZeroRows) * kPitch);
  float* blob = reinterpret_cast<float*>(&sm + 1);  // the staged small weights (TowerNet::blob prefix)

  const int HW = H * W;
  const int b0 = blockIdx.x * bpw;
  if (b0 >= n) return;  // block-uniform
  const int nbrd = min(bpw, n - b0);
  const int live = nbrd * HW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int zrow = TR;
  T16_RSTAMP(22);
  T16_STAMP(0);
  // the alternative tile height of a dual launch: a slot plan and an LDS
  // staging of its own
  const bool alt = 16 * MBT != T.tile_rows && 16 * MBT == T.alt_rows;
  const bool wpd_lds = alt ? T.alt_wpd_lds : T.wpd_lds;
  const bool wv1_lds = alt ? T.alt_wv1_lds : T.wv1_lds;
  // (the alternative tiles' staged value dense wv1 -- 43 KB at Connect-4 --
  // arrives during the last conv2, as wv1_xt's does: at the kernel's start
  // it would queue ahead of the slot plan's and the boards' loads)
  const bool wv1_late = alt && wv1_lds;
  // small weights into LDS, in the background of the stem
  dma_to_lds<NT>(reinterpret_cast<uint4*>(blob), T.blob,
                 (wv1_late ? T.off_wv1 : alt ? T.alt_staged_floats : T.staged_floats) / 4, wave, lane);
  for (int i = tid; i < kZeroRows * kPitch / 16; i += NT) act[zrow * kPitch / 16 + i] = make_uint4(0u, 0u, 0u, 0u);
  if (tid < 2) sm.flag[tid] = 0;  // published by the barrier after the stem's MFMAs

  const int mh = wave % NWM, nq = wave / NWM, r16 = lane & 15, gq = lane >> 4;
  // a lane's slots r0 + 16 mb and their pixel words: the slot plan's
  // (T.slot_pix, a full tile's boards; the boards past this tile's are
  // emptied, keeping their rows' bank residues) or the natural order
  const int r0 = mh * MBW * 16 + r16;
  int yx[MBW];
  // (the plan is for the TowerNet's tile height: a smaller tile of the same
  // boards -- chess's 64-row tiles -- runs in natural order, the same bits)
  const bool planned = 16 * MBT == T.tile_rows || alt;
  // wv1 staged behind X's dead tile only in the tile height it was sized for
  // (tower16_wv1_xtile_fits); another tile height reads it from L2
  const bool wv1_xt = T.wv1_xtile && 16 * MBT == T.tile_rows;
  const int* plan = !planned ? nullptr : alt ? T.alt_slot_pix : T.slot_pix;
  T16_STAMP(56);
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    const int rr = r0 + 16 * mb;
    if (plan) {
      const int v = *gbl(plan + rr);
      yx[mb] = pix_ok(v) && (v >> 16) >= nbrd ? (127 << 8) | (pix_row(v, HW, W) & 7) : v;
    } else {
      const bool valid = rr < live;
      const int b = valid ? rr / HW : 0;
      const int p = rr - b * HW;
      yx[mb] = valid ? (b << 16) | ((p / W) << 8) | (p - (p / W) * W) : (127 << 8) | (rr & 7);
    }
  }
  // this wave's tap skips (2 bits per tap over its blocks 0 and 1)
  // (chess's 64-row tiles never run the plan: a compile-time 0 there, so
  // each tap compiles to one body instead of three)
  const int skw = (ROWS && 16 * MBT != 128) ? 0 : !planned ? 0 : alt ? T.alt_skip[mh] : T.skip[mh];
  const int cq0 = 8 * nq + gq;  // channel quad of a lane's N block 0 (block 1: + 4)
  // double-buffered: one accumulator set (conv2 runs the block's 1x1
  // projection residual first, from X, which nothing overwrites before its
  // epilogue); in place: the residual is taken in conv1's phase (X is then
  // overwritten by conv1's output) into a second set accr
  t_f4 acc[MBW][2], accr_[MBW][2];
  auto& accr = DB ? acc : accr_;
  float4 yv[2 * MBW];

  // ---------------------------------------------------------------- stem
  if constexpr (ROWS) {
    // input rows -> H's tile (512 B split16 per pixel: t0 copied, t1 from the
    // rows' x 2^12 scale to the tower's unscaled term), then the stem conv
    // (F -> F over the padded input channels) as a K loop into X
    char* dst = reinterpret_cast<char*>(bufH);
    // the second term's x 2^12 scale (rows) -> the tower's unscaled term
    auto t1_unscale = [](uint32_t w) {
      const az_h2 h = __builtin_bit_cast(az_h2, w);
      return pk_f16((float)h[0] * 0x1p-12f, (float)h[1] * 0x1p-12f);
    };
    if (lv.leaf) {
      // planes 64-127 of each pixel from the board's queued leaf (chess
      // self-play, first_chunk 2: planes 0-63 are never read), the float4s
      // encode_queue_kernel would have stored, split and unscaled alike
      const azc::Pos st = azc::start_pos();
      for (int i = tid; i < live * 16; i += NT) {
        const int rr = i >> 4, c4 = 16 + (i & 15), b = rr / HW, pix = rr - b * HW;
        const int s = *gbl(lv.eval_slot + b0 + b);
        const azc::Pos cur = azc::load_pos(static_cast<const az_chess_pos*>(lv.leaf)[s]);
        const bool initial = *gbl(lv.path_len + s) == 0 && *gbl(lv.initial + s) != 0;
        float f[6], v[4];
        azc::state_feats(cur, f);
        azc::full_state4(st, cur, initial, f, pix, 4 * c4, v);
        uint2 t0, t1;
        split16x4(make_float4(v[0], v[1], v[2], v[3]), t0, t1);
        char* q = dst + rr * kPitch;
        *reinterpret_cast<uint2*>(q + 8 * c4) = t0;
        *reinterpret_cast<uint2*>(q + 256 + 8 * c4) = make_uint2(t1_unscale(t1.x), t1_unscale(t1.y));
      }
    } else {
      const uint4* src = rows + (size_t)b0 * HW * 32;
#pragma unroll 4
      for (int i = tid; i < live * 32; i += NT) {
        uint4 v = gld(src + i);
        if ((i & 31) >= 16) v = make_uint4(t1_unscale(v.x), t1_unscale(v.y), t1_unscale(v.z), t1_unscale(v.w));
        *reinterpret_cast<uint4*>(dst + (i >> 5) * kPitch + (i & 31) * 16) = v;
      }
    }
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = t_f4{0.f, 0.f, 0.f, 0.f};
    __builtin_amdgcn_s_waitcnt(0);  // this wave's blob DMA pieces have landed ...
    __syncthreads();                // ... every wave's, and the input rows
    if (first_chunk == 2) AZ_KLOOP<MBW, 0, 2>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, skw);
    else AZ_KLOOP<MBW, 0, 0>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, skw);
    if (!dbuf) __syncthreads();  // in place: every wave is done reading the input before X overwrites it
  } else {
  // conv3x3 4 -> F + folded BN + ReLU on the MFMA: k = tap*4 + plane (36 of
  // two 32-wide k-steps), the im2col operand built in registers from the
  // boards' bits (one-hot planes [empty, own, opp, 1], board.py:83-98: exact
  // in fp16, second term 0) or from x split into two fp16 terms -- for a
  // one-hot x the operands, and so the outputs, are bitwise the boards'.
  {
    // both k-steps' weight fragments and each M block's board (global loads
    // issued together: one latency, no barrier before the MFMAs)
    const uint4* ws = T.stem16 + (size_t)(nq * 2) * 2 * 64 + lane;
    uint4 bs2[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int q = 0; q < 4; ++q) bs2[ks][q] = gld(ws + (size_t)ks * 1024 + q * 64);
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = t_f4{0.f, 0.f, 0.f, 0.f};
    // M blocks in groups of at most 4 (a group's boards and operands in registers)
    constexpr int SG = MBW <= 4 ? MBW : MBW % 4 == 0 ? 4 : MBW % 3 == 0 ? 3 : 1;
    static_assert(MBW % SG == 0, "stem groups");
#pragma unroll
    for (int g0 = 0; g0 < MBW; g0 += SG) {
      Board bd[SG];
      if (boards) {
#pragma unroll
        for (int i = 0; i < SG; ++i) bd[i] = gld(boards + b0 + (yx[g0 + i] >> 16));
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const uint4(&bs)[4] = bs2[ks];
        const t_h8 B0[2] = {__builtin_bit_cast(t_h8, bs[0]), __builtin_bit_cast(t_h8, bs[2])};
        const t_h8 B1[2] = {__builtin_bit_cast(t_h8, bs[1]), __builtin_bit_cast(t_h8, bs[3])};
#pragma unroll
        for (int i = 0; i < SG; ++i) {
          const int mb = g0 + i;
          float v[8];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int t = 8 * ks + 2 * gq + h;  // tap of k = 32 ks + 8 gq + 4 h + plane
            const int dy = t / 3 - 1, dx = t - (t / 3) * 3 - 1;
            const int py = (yx[mb] >> 8) & 255, px = yx[mb] & 255;
            const bool ok = t < 9 && py + dy >= 0 && py + dy < H && px + dx >= 0 && px + dx < W;
            float4 pl = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ok) {
              const int q = (py + dy) * W + px + dx;
              if (boards) {
                const uint64_t ow = q < 64 ? bd[i].own[0] : bd[i].own[1],
                               op = q < 64 ? bd[i].opp[0] : bd[i].opp[1];
                const bool o = (ow >> (q & 63)) & 1ull, e = (op >> (q & 63)) & 1ull;
                pl = make_float4(o || e ? 0.f : 1.f, o ? 1.f : 0.f, e ? 1.f : 0.f, 1.f);
              } else {
                pl = gld(x + (size_t)(b0 + (yx[mb] >> 16)) * HW + q);
              }
            }
            v[4 * h + 0] = pl.x;
            v[4 * h + 1] = pl.y;
            v[4 * h + 2] = pl.z;
            v[4 * h + 3] = pl.w;
          }
          uint4 a0, a1;
          split_u8(v, a0, a1);
          // t1*B0 + t0*b1 + t0*B0 per N block, as the K loop's k-step
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) {
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], __builtin_bit_cast(t_h8, a1), acc[mb][nb], 0, 0, 0);
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B1[nb], __builtin_bit_cast(t_h8, a0), acc[mb][nb], 0, 0, 0);
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(B0[nb], __builtin_bit_cast(t_h8, a0), acc[mb][nb], 0, 0, 0);
          }
        }
      }
    }
  }
  T16_STAMP(57);
  __builtin_amdgcn_s_waitcnt(0);  // this wave's blob DMA pieces have landed ...
  T16_STAMP(58);
  __syncthreads();                // ... and every wave's: the blob is readable
  }  // !ROWS
  T16_STAMP(1);
  {
    const float osc = ROWS ? T.stem_ks : T.stem_s;
    const float* bb = blob + T.off_stemb;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const float4 bc = *reinterpret_cast<const float4*>(bb + 32 * nq + 16 * nb + 4 * gq);
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        const t_f4 a = acc[mb][nb];
        yv[mb * 2 + nb] = make_float4(fmaxf(fmaf(a[0], osc, bc.x), 0.f), fmaxf(fmaf(a[1], osc, bc.y), 0.f),
                                      fmaxf(fmaf(a[2], osc, bc.z), 0.f), fmaxf(fmaf(a[3], osc, bc.w), 0.f));
      }
    }
  }
  int par = 0;
  // scale state: buffer contents X (block input) and H (conv1 output)
  bool anyX = store_layer<MBW>(bufX, HW, W, yx, cq0, yv, sm, par, sm.sc[0], nbrd, err);
  bool anyH = false;
  float* red = nullptr;  // the heads' 1x1 partials [TR][16][3] (set by the last block)
  const int J = T.hidden;  // value head hidden units
  par ^= 1;
  T16_STAMP(21);

  // ---------------------------------------------------------------- tower
  const int depth = T.depth;
  for (int d = 0; d < depth; ++d) {
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        acc[mb][nb] = t_f4{0.f, 0.f, 0.f, 0.f};
        accr_[mb][nb] = t_f4{0.f, 0.f, 0.f, 0.f};
      }
    // conv1, input X (in place: + the projection residual into accr)
    T16_WSTAMP(d, 0);
    if constexpr (DB) AZ_KLOOP<MBW, 0, 0>(bufX, T.k1[d], nullptr, acc, acc, yx, H, W, zX, nq, lane, skw);
    else AZ_KLOOP<MBW, 4, 0>(bufX, T.k1[d], T.k2[d], acc, accr_, yx, H, W, zX, nq, lane, skw);
    T16_WSTAMP(d, 1);
    if (d < 4) T16_STAMP(2 + 4 * d);
    if (d < 4) T16_STAMP4(24 + 4 * d);
    if (!dbuf) __syncthreads();  // in place: every wave is done reading X before H overwrites it
    if (d < 4) T16_STAMP(40 + d);
    {
      const float osc = T.s1[d];
      const float* bb = blob + T.off_b1 + d * 128;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const float4 bc = *reinterpret_cast<const float4*>(bb + 32 * nq + 16 * nb + 4 * gq);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          const float o = anyX ? ldexpf(osc, sm.sc[0][yx[mb] >> 16]) : osc;
          const t_f4 a = acc[mb][nb];
          yv[mb * 2 + nb] = make_float4(fmaxf(fmaf(a[0], o, bc.x), 0.f), fmaxf(fmaf(a[1], o, bc.y), 0.f),
                                        fmaxf(fmaf(a[2], o, bc.z), 0.f), fmaxf(fmaf(a[3], o, bc.w), 0.f));
        }
      }
    }
    anyH = store_layer<MBW>(bufH, HW, W, yx, cq0, yv, sm, par, sm.sc[1], nbrd, err);
    par ^= 1;
    if (d < 4) T16_STAMP(3 + 4 * d);
    // the residual was accumulated at X's scale, conv2 runs at H's
    auto rescale = [&]() {
      if (anyX || anyH) {
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          const int e = (anyX ? sm.sc[0][yx[mb] >> 16] : 0) - (anyH ? sm.sc[1][yx[mb] >> 16] : 0);
          if (e) {
            const float f = ldexpf(1.f, e);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) accr[mb][nb] *= f;
          }
        }
      }
    };
    T16_WSTAMP(d, 2);
    if constexpr (DB) {
      // conv2: the 1x1 projection residual from X's rows, then (once every
      // wave is past them: X's tile is dead from here) the taps on H; the last
      // block streams the value dense's wv1 into X's tile behind the heads'
      // partials while the taps run (every wave a share).  The same sums in
      // the same order as the in-place form: bitwise the same outputs
      const bool wv1x = (wv1_xt || wv1_late) && d + 1 == depth;  // read before the K loop's asm ("memory")
      auto mid = [&]() {
        rescale();
        __syncthreads();
        if (wv1x)
          dma_to_lds<NT>(reinterpret_cast<uint4*>(wv1_xt ? reinterpret_cast<float*>(bufX) + TR * 48 : blob + T.off_wv1),
                         T.blob + T.off_wv1, HW * J / 4, wave, lane);
      };
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = t_f4{0.f, 0.f, 0.f, 0.f};  // conv1's sums are stored
      AZ_KLOOP<MBW, 4, 0>(bufH, T.k2[d], T.k2[d], acc, acc, yx, H, W, zH, nq, lane, skw, -(TR + kZeroRows),
                            mid);
    } else {
      rescale();
      // conv2 on H, on top of the residual
      AZ_KLOOP<MBW, 0, 0>(bufH, T.k2[d], nullptr, accr, accr, yx, H, W, zH, nq, lane, skw);
    }
    T16_WSTAMP(d, 3);
    if (d < 4) T16_STAMP(4 + 4 * d);
    if (d < 4) T16_STAMP4(26 + 4 * d);
    const float osc = T.s2[d];
    const float* bb = blob + T.off_b2 + d * 128;
    if (d + 1 < depth) {
      if (!dbuf) __syncthreads();  // in place: every wave is done reading H
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const float4 bc = *reinterpret_cast<const float4*>(bb + 32 * nq + 16 * nb + 4 * gq);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
          const float o = anyH ? ldexpf(osc, sm.sc[1][yx[mb] >> 16]) : osc;
          const t_f4 a = accr[mb][nb];
          yv[mb * 2 + nb] = make_float4(fmaxf(fmaf(a[0], o, bc.x), 0.f), fmaxf(fmaf(a[1], o, bc.y), 0.f),
                                        fmaxf(fmaf(a[2], o, bc.z), 0.f), fmaxf(fmaf(a[3], o, bc.w), 0.f));
        }
      }
      anyX = store_layer<MBW>(bufX, HW, W, yx, cq0, yv, sm, par, sm.sc[0], nbrd, err);
      par ^= 1;
      if (d < 4) T16_STAMP(5 + 4 * d);
      continue;
    }
    // ------------------------------------------------------------ heads
    // last block: its output goes straight into the 1x1 head convs (policy
    // F -> 2, value F -> 1, folded BN, ReLU; model.py:68-149): per lane the
    // partial sums over its 8 channels, to LDS as 16 partials per pixel (no
    // cross-lane step), summed in a fixed order below.  Double-buffered, they
    // go to X's tile (dead since conv1's barrier) while other waves still
    // read H; in place, after a barrier.
    if (dbuf) {
      red = reinterpret_cast<float*>(bufX);  // (wv1 behind them since the start of this conv2)
    } else {
      __syncthreads();
      red = reinterpret_cast<float*>(act);
    }
    const float* wpc = blob + T.off_wpc;
    const float* wvc = blob + T.off_wvc;
    int hr[MBW], hyx[MBW], hb[MBW];  // laundered (see k_loop): addresses recomputed here, not hoisted and spilled
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      hr[mb] = pix_row(yx[mb], HW, W);
      hyx[mb] = yx[mb];
      hb[mb] = yx[mb] >> 16;
      asm volatile("" : "+v"(hr[mb]), "+v"(hyx[mb]), "+v"(hb[mb]));
    }
    int hq = 32 * nq + 4 * gq;  // the lane's first channel (N block 0)
    asm volatile("" : "+v"(hq));
    T16_STAMP4(48);
    // the lane's 8 channels' bias and head weights, read once (the partial
    // stores below could alias them, so per M block they would be re-read)
    float bcv[2][4], wp[2][4][2], wv[2][4];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int c0 = hq + 16 * nb;
      const float4 bc = *reinterpret_cast<const float4*>(bb + c0);
      const float4 p01 = *reinterpret_cast<const float4*>(wpc + 2 * c0);      // channels c0, c0+1
      const float4 p23 = *reinterpret_cast<const float4*>(wpc + 2 * c0 + 4);  // c0+2, c0+3
      const float4 vv = *reinterpret_cast<const float4*>(wvc + c0);
      const float bq[4] = {bc.x, bc.y, bc.z, bc.w}, pq[8] = {p01.x, p01.y, p01.z, p01.w, p23.x, p23.y, p23.z, p23.w},
                  vq[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        bcv[nb][v] = bq[v];
        wp[nb][v][0] = pq[2 * v];
        wp[nb][v][1] = pq[2 * v + 1];
        wv[nb][v] = vq[v];
      }
    }
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      T16_STAMP4(49 + mb);
      const float o = anyH ? ldexpf(osc, sm.sc[1][hb[mb]]) : osc;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float yy = fmaxf(fmaf(accr[mb][nb][v], o, bcv[nb][v]), 0.f);
          a0 = fmaf(yy, wp[nb][v][0], a0);
          a1 = fmaf(yy, wp[nb][v][1], a1);
          a2 = fmaf(yy, wv[nb][v], a2);
        }
      }
      if (pix_ok(hyx[mb])) {
        float* q = red + (hr[mb] * 16 + nq * 4 + gq) * 3;
        q[0] = a0;
        q[1] = a1;
        q[2] = a2;
      }
    }
  }
  T16_STAMP4(54);
  T16_STAMP(42);
  T16_STAMP4(43);
  if (wv1_xt || wv1_late) __builtin_amdgcn_s_waitcnt(0);  // this wave's wv1 DMA pieces have landed ...
  __syncthreads();  // ... the partials are complete; no activation row is read any more
  T16_STAMP(18);
  if constexpr (ROWS) {
    // per pixel (policy 0, policy 1, value) = 16 partials in order + folded
    // bias, ReLU: the dense heads read them (az_nn.hip policy_dense_kernel,
    // heads_tail_kernel)
    const float* hbias = blob + T.off_hb;
    const float bpc0 = hbias[0], bpc1 = hbias[1], bvc0 = hbias[2];
    for (int rr = tid; rr < live; rr += NT) {
      const float* q = red + rr * 48;
      float t[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) t[k] += q[3 * j + k];
      feat[(size_t)b0 * HW + rr] =
          make_float4(fmaxf(t[0] + bpc0, 0.f), fmaxf(t[1] + bpc1, 0.f), fmaxf(t[2] + bvc0, 0.f), 0.f);
    }
    return;
  }

  // head scratch (H's tile, or the in-place tile past the partials): the
  // flattened features per board (Keras Flatten of NHWC: [p][c]) pf [bpw][2HW]
  // and, pixel-major for the value dense's reads, vf [HW][8 boards]; logits
  // lg [bpw][A], policy partials pp [NT], value partials vp [bpw][P][J],
  // value hidden units hv [bpw][J]
  const int P = NT / J;
  float* pf = dbuf ? reinterpret_cast<float*>(bufH) : red + TR * 48;
  float* vf = pf + ((bpw * 2 * HW + 3) & ~3);  // 16-byte aligned
  float* lg = vf + kTowerMaxBoards * HW;
  float* pp = lg + bpw * A;
  float* vp = pp + NT;
  float* hv = vp + bpw * P * J;
  {
    const float* hbias = blob + T.off_hb;
    const float bpc0 = hbias[0], bpc1 = hbias[1], bvc0 = hbias[2];
    for (int i = tid; i < 3 * live; i += NT) {  // (pixel row, output) pairs; 16 partials in order
      const int rr = i / 3, k = i - 3 * rr;
      const float* q = red + rr * 48 + k;
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) t += q[3 * j];
      const int b = rr / HW, p = rr - b * HW;
      if (k < 2) pf[b * 2 * HW + 2 * p + k] = fmaxf(t + (k ? bpc1 : bpc0), 0.f);
      else vf[p * kTowerMaxBoards + b] = fmaxf(t + bvc0, 0.f);
    }
  }
  __syncthreads();
  T16_STAMP(44);
  // policy Dense(A): 16 threads per logit, each a strided slice of the 2HW
  // features, then the 16 partials in order; value Dense(J): P threads per
  // hidden unit, each a strided slice of the pixels for every board, then
  // the P partials in order
  {
    const int K = 2 * HW, O = nbrd * A, OP = NT / 16;
    const float* bpd = blob + T.off_bpd;
    const float* bv1 = blob + T.off_bv1;
    const float* wv2 = blob + T.off_wv2;
    auto policy_part = [&](int base, auto wpd) {
      const int o = base + tid / 16, pi = tid & 15;
      float sacc = 0.f;
      if (o < O) {
        const int b = o / A, a = o - b * A;
        const float* pb = pf + b * K;
        for (int k0 = pi; k0 < K; k0 += 64) {  // 4 features per batch, their reads ahead of the FMAs
          float xv[4], wv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int k = k0 + 16 * u;
            xv[u] = k < K ? pb[k] : 0.f;
            wv[u] = k < K ? wpd[k * A + a] : 0.f;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) sacc = fmaf(xv[u], wv[u], sacc);
        }
      }
      pp[tid] = sacc;
    };
    // NBV: the boards a pass covers, 4 when the tile holds at most 4 (C4: 3)
    // -- the per-board sums are the same either way, the 8-board form spent
    // 5/8 of its FMAs on boards the tile does not have
    auto value_part_n = [&](auto wv1, auto nbv) {
      constexpr int NBV = decltype(nbv)::value;
      const int j = tid % J, q = tid / J;  // q: wave-uniform for J >= 64
      if (q >= P) return;
      float sv[NBV];
#pragma unroll
      for (int b = 0; b < NBV; ++b) sv[b] = 0.f;
      for (int p0 = q; p0 < HW; p0 += 4 * P) {  // 4 pixels per batch, every read ahead of the FMAs
        float w[4], v[4][NBV];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int p = p0 + u * P;
          const int pc = p < HW ? p : 0;
          w[u] = p < HW ? wv1[pc * J + j] : 0.f;
          // the pixel's boards (past nbrd: stale scratch, never stored)
#pragma unroll
          for (int h = 0; h < NBV / 4; ++h) {
            const float4 f = *reinterpret_cast<const float4*>(vf + pc * kTowerMaxBoards + 4 * h);
            v[u][4 * h] = f.x, v[u][4 * h + 1] = f.y, v[u][4 * h + 2] = f.z, v[u][4 * h + 3] = f.w;
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int b = 0; b < NBV; ++b) sv[b] = fmaf(v[u][b], w[u], sv[b]);
      }
#pragma unroll
      for (int b = 0; b < NBV; ++b)
        if (b < nbrd) vp[(b * P + q) * J + j] = sv[b];
    };
    auto value_part = [&](auto wv1) {
      if (nbrd <= 4) value_part_n(wv1, IC<4>{});
      else value_part_n(wv1, IC<kTowerMaxBoards>{});
    };
    for (int base = 0;; base += OP) {  // block-uniform
      if (wpd_lds) policy_part(base, blob + T.off_wpd);
      else policy_part(base, gbl(T.blob + T.off_wpd));
      if (base == 0) {
        if (wv1_lds) value_part(blob + T.off_wv1);
        else if (wv1_xt) value_part(reinterpret_cast<const float*>(bufX) + TR * 48);
        else value_part(gbl(T.blob + T.off_wv1));
      }
      if (base == 0) T16_STAMP(45);
      __syncthreads();
      if (base == 0) T16_STAMP(46);
      if (tid < OP && base + tid < O) {
        const int o = base + tid, a = o % A;
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) t += pp[tid * 16 + j];
        lg[o] = t + bpd[a];
      }
      if (base == 0) {
        for (int i = tid; i < nbrd * J; i += NT) {
          const int b = i / J, j = i - b * J;
          float t = 0.f;
          for (int q = 0; q < P; ++q) t += vp[(b * P + q) * J + j];
          hv[i] = fmaxf(t + bv1[j], 0.f) * wv2[j];
        }
      }
      if (base == 0) T16_STAMP(47);
      __syncthreads();
      if (base + OP >= O) break;
    }
  }
  // softmax (one wave per board) and tanh
  const float bv2 = blob[T.off_hb + 3];
  for (int b = wave; b < nbrd; b += NT / 64) {  // wave-uniform
    float m = -INFINITY;
    for (int a = lane; a < A; a += 64) m = fmaxf(m, lg[b * A + a]);
    m = wmax(m);
    float z = 0.f;
    for (int a = lane; a < A; a += 64) z += expf(lg[b * A + a] - m);
    z = wsum(z);
    for (int a = lane; a < A; a += 64) probs[(size_t)(b0 + b) * A + a] = expf(lg[b * A + a] - m) / z;
    float v = 0.f;
    for (int j = lane; j < J; j += 64) v += hv[b * J + j];
    v = wsum(v);
    if (lane == 0) values[b0 + b] = tanhf(v + bv2);
  }
  T16_STAMP(19);
  T16_RSTAMP(23);
}

template <int MBT, int NWM, bool ROWS, bool DB>
__global__ __launch_bounds__(NWM * 256, NWM) void tower16_kernel(const TowerNet* __restrict__ net,
                                                               const Board* __restrict__ boards,
                                                               const float4* __restrict__ x,
                                                               const uint4* __restrict__ rows,
                                                               const int* __restrict__ count, int n_static,
                                                               int H, int W, int A, int bpw,
                                                               float* __restrict__ probs,
                                                               float* __restrict__ values,
                                                               float4* __restrict__ feat, int first_chunk,
                                                               unsigned long long* __restrict__ err,
                                                               TowerLeaves lv) {
  tower16_tile<MBT, NWM, ROWS, DB>(net, boards, x, rows, count ? *count : n_static, H, W, A, bpw, probs, values,
                                   feat, first_chunk, err, lv);
}

// One launch, two tile heights, chosen on the device by the live board count
// (the host enqueues the launch before the select that fills the queue has
// run): a launch of at most T.alt_max_boards boards runs the alternative,
// shorter tiles (Connect-4: 96 rows of two boards instead of 128 rows of
// three -- 3 M blocks per wave instead of 4, so a tile's latency drops by a
// quarter), a larger one the primary tiles (fewer weight passes; the
// shorter tiles' 1.5x tiles would outnumber the CUs).  With the LRU
// transposition cache a Connect-4 lane evaluates ~120 boards per simulation
// and the step is bound by each lane's chain of launches: +4.4% games/s
// (profiles/r6/ab_t96.txt); at 373 / 1113 boards the shorter tiles lose 20%
// (ab_t96off.txt, ab_t96s400.txt).  Grid: the alternative's tiles; the
// primary's blocks past its tiles leave at once.  Every board's outputs are
// the same bits in either tile (batch invariance, the slot plans' bitwise
// order).
template <int MBT, int MBT2, bool DB>
__global__ __launch_bounds__(512, 2) void tower16_dual_kernel(const TowerNet* __restrict__ net,
                                                              const Board* __restrict__ boards,
                                                              const float4* __restrict__ x,
                                                              const int* __restrict__ count, int n_static,
                                                              int H, int W, int A, int bpw, int bpw2,
                                                              float* __restrict__ probs, float* __restrict__ values,
                                                              unsigned long long* __restrict__ err) {
  const int n = count ? *count : n_static;
  if (n <= net->alt_max_boards)  // uniform over the launch
    tower16_tile<MBT2, 2, false, DB>(net, boards, x, nullptr, n, H, W, A, bpw2, probs, values, nullptr, 0, err, {});
  else
    tower16_tile<MBT, 2, false, DB>(net, boards, x, nullptr, n, H, W, A, bpw, probs, values, nullptr, 0, err, {});
}

}  // namespace

#ifdef AZ_T16_STAMPS
}  // namespace az
extern "C" int az_t16_stamps(unsigned long long* out) {  // [4096][24] of the last launch(es)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(az::g_t16_stamps), sizeof(az::g_t16_stamps)) == hipSuccess ? 0 : -1;
}
extern "C" int az_t16_wstamps(unsigned long long* out) {  // [4096][8][5]
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(az::g_t16_wstamps), sizeof(az::g_t16_wstamps)) == hipSuccess ? 0 : -1;
}
namespace az {
#endif

int tower16_tile_rows(int HW) {
  if (HW > 128) return 0;
  // boards of 65-96 pixels (9x9): 192-row tiles of two boards (in place: two
  // such tiles exceed the LDS), which halve the weight stream per board --
  // round 5, configs[2]: 73.1 -> 81.3 games/s (profiles/r5/ab_9x9.txt)
  if (HW > 64 && HW <= 96) return 192;
  // 128-row tiles unless 96 rows hold the same boards (more rows per tile, same work per board)
  const int b128 = std::min(128 / HW, kTowerMaxBoards), b96 = std::min(96 / HW, kTowerMaxBoards);
  if (b96 >= 1 && b96 * HW * 128 >= b128 * HW * 96) return 96;  // 96-row tiles are at least as full
  return 128;
}

int tower16_boards_per_tile(int HW, int tr) { return tr ? std::min(tr / HW, kTowerMaxBoards) : 0; }

size_t tower16_lds_bytes(int HW, int tr, int staged_floats, bool dbuf) {
  (void)HW;
  return (size_t)((dbuf ? 2 : 1) * tr + kZeroRows) * kPitch + sizeof(TowerSmem) + (size_t)staged_floats * sizeof(float);
}

bool tower16_heads_fit(int HW, int tr, int A, int hidden, bool dbuf) {
  // the kernel's head scratch (pf, vf, lg, pp, vp, hv) behind the partials
  // (in place) or in H's tile (double-buffered), for the larger block size
  const int bpw = tower16_boards_per_tile(HW, tr), nt = 512;
  if (!tr || hidden < 1 || hidden > 256) return false;
  const int p = nt / hidden;
  const size_t need = (size_t)bpw * 2 * HW + 3 + (size_t)kTowerMaxBoards * HW + (size_t)bpw * A + nt +
                      (size_t)bpw * p * hidden + (size_t)bpw * hidden;
  const size_t have = (size_t)tr * (kPitch / 4) - (dbuf ? 0 : (size_t)tr * 48);
  return need <= have;
}

bool tower16_wv1_xtile_fits(int HW, int tr, int hidden) {
  return tr && (HW * hidden) % 4 == 0 && (size_t)tr * 48 * 4 + (size_t)HW * hidden * 4 <= (size_t)tr * kPitch;
}

// The slot plan (192-, 128- and 96-row tiles, 8 waves: M half h = blocks
// (tr / 32) h ..).
// A 3x3 'same' conv tap (dy, dx) reads zeros for every pixel on the board edge
// it points past; a block whose 16 slots all hold such pixels (or are empty)
// would add exact zeros for that tap, so it skips the tap's MFMAs and reads.
// Border blocks: half 0 = [top (y = 0: skips dy = -1), bottom (dy = +1), 2
// interior], half 1 = [left (x = 0: dx = -1), right (dx = +1), 2 interior]:
// each wave skips 6 of its 36 block-taps per conv (C4: 3 boards, 16.7% of the
// 3x3 MFMAs).  A tile with too few edge pixels for four border blocks (one
// 9x9 board in a 96-row tile) gets top | bottom only, filled up with pads
// (11% of the 3x3 MFMAs).  Bank conflicts: a ds_read_b128 lane group
// reads 8 slots of one term parity ({0-3, 12-15} or {4-11}) at one tap shift;
// its bank quads are 2 row + slot (mod 16), so the 8 slots' LDS rows must
// differ mod 8.  Per residue r the pixels with row = r (mod 8) fill 2 slots of
// each border block (a bipartite matching against the edge classes; corners
// belong to two), then 2 of each interior block; an interior residue past 8
// takes a free slot (one 2-way conflict).
namespace {
struct PlanBorder {
  int cls, blk;  // edge class (0 top, 1 left, 2 bottom, 3 right), tile block
};

// one layout of border blocks: false when a border pad leaves a pixel without
// a slot or a border block would hold fewer than 8 edge pixels
bool slot_plan_try(int H, int W, int tr, const std::vector<PlanBorder>& borders, std::vector<int>& slot_pix,
                   int skip[2]) {
  const int HW = H * W, nb = tower16_boards_per_tile(HW, tr), nblk = tr / 16, half = nblk / 2;
  auto cls = [&](int y, int x, int c) {
    return c == 0 ? y == 0 : c == 1 ? x == 0 : c == 2 ? y == H - 1 : x == W - 1;
  };
  const int nbor = (int)borders.size();
  std::vector<int> interior;
  for (int k = 0; k < nblk; ++k) {
    bool b = false;
    for (const PlanBorder& e : borders) b = b || e.blk == k;
    if (!b) interior.push_back(k);
  }
  const int nint = (int)interior.size();
  const int S1[8] = {0, 1, 2, 3, 12, 13, 14, 15}, S2[8] = {4, 5, 6, 7, 8, 9, 10, 11};
  const int kEmpty = 127 << 8;
  std::vector<int> slot(tr, -1);  // pixel word, or <= -2: free (residue -2 - v)
  auto word = [&](int n) { return ((n / HW) << 16) | (((n % HW) / W) << 8) | (n % W); };
  std::vector<int> overflow;
  for (int r = 0; r < 8; ++r) {
    std::vector<int> P;  // natural rows with residue r
    for (int n = r; n < nb * HW; n += 8) P.push_back(n);
    // border slots: border e, copy k (0, 1); Kuhn's matching of the residue's edge pixels
    const int ns = 2 * nbor;
    std::vector<int> owner(ns, -1);
    std::function<bool(int, std::vector<char>&)> aug = [&](int pi, std::vector<char>& seen) {
      const int n = P[pi], y = (n % HW) / W, x = n % W;
      for (int sl = 0; sl < ns; ++sl) {
        if (seen[sl] || !cls(y, x, borders[sl / 2].cls)) continue;
        seen[sl] = 1;
        if (owner[sl] < 0 || aug(owner[sl], seen)) {
          owner[sl] = pi;
          return true;
        }
      }
      return false;
    };
    for (int pi = 0; pi < (int)P.size(); ++pi) {
      std::vector<char> seen(ns, 0);
      aug(pi, seen);
    }
    std::vector<char> used(P.size(), 0);
    for (int sl = 0; sl < ns; ++sl) {
      const int at = borders[sl / 2].blk * 16 + ((sl & 1) ? S2[r] : S1[r]);
      if (owner[sl] >= 0) {
        slot[at] = word(P[owner[sl]]);
        used[owner[sl]] = 1;
      } else {
        slot[at] = kEmpty | r;  // a pad: reads zero rows at its residue
      }
    }
    // interior: 2 per block at this residue's positions, in order
    int k = 0;
    for (int pi = 0; pi < (int)P.size(); ++pi) {
      if (used[pi]) continue;
      if (k < 2 * nint) {
        slot[interior[k / 2] * 16 + ((k & 1) ? S2[r] : S1[r])] = word(P[pi]);
        ++k;
      } else {
        overflow.push_back(P[pi]);
      }
    }
    for (; k < 2 * nint; ++k) slot[interior[k / 2] * 16 + ((k & 1) ? S2[r] : S1[r])] = -2 - r;
  }
  // overflow pixels into free interior slots (one 2-way bank conflict each)
  for (int n : overflow) {
    bool placed = false;
    for (int j = 0; j < tr && !placed; ++j)
      if (slot[j] <= -2) {
        slot[j] = word(n);
        placed = true;
      }
    if (!placed) return false;  // the border pads took the slots a pixel needs
  }
  for (int j = 0; j < tr; ++j)
    if (slot[j] <= -2) slot[j] = kEmpty | (-2 - slot[j]);
  for (const PlanBorder& e : borders) {
    int px = 0;
    for (int j = 0; j < 16; ++j) px += ((slot[e.blk * 16 + j] >> 8) & 255) != 127;
    if (px < 8) return false;
  }
  skip[0] = skip[1] = 0;
  for (const PlanBorder& e : borders) {
    const int h = e.blk / half, bit = e.blk % half;
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3 - 1, dx = t % 3 - 1;
      const bool past = e.cls == 0 ? dy == -1 : e.cls == 1 ? dx == -1 : e.cls == 2 ? dy == 1 : dx == 1;
      if (past) skip[h] |= (1 << bit) << (2 * t);
    }
  }
  for (int h = 0; h < 2; ++h)  // the kernel's tap bodies skip one block per tap (masks 0, 1, 2)
    for (int t = 0; t < 9; ++t)
      if (((skip[h] >> (2 * t)) & 3) == 3) skip[h] &= ~(2 << (2 * t));
  slot_pix = slot;
  return true;
}
}  // namespace

void tower16_slot_plan(int H, int W, int tr, std::vector<int>& slot_pix, int skip[2]) {
  slot_pix.clear();
  skip[0] = skip[1] = 0;
  if ((tr != 192 && tr != 128 && tr != 96) || H < 3 || W < 3 || !tower16_boards_per_tile(H * W, tr)) return;
  const int half = tr / 32;
  // layouts in order: T, B | L, R; then top | bottom (e.g. one 9x9 board in a
  // 96-row tile: too few edge pixels for four blocks)
  const std::vector<std::vector<PlanBorder>> layouts = {
      {{0, 0}, {2, 1}, {1, half}, {3, half + 1}},
      {{0, 0}, {2, half}}};
  for (const auto& borders : layouts)
    if (slot_plan_try(H, W, tr, borders, slot_pix, skip)) return;
  skip[0] = skip[1] = 0;
}

double tower16_issued_flop_per_board(int HW, int tr, int depth, const int skip[2], bool rows_stem, int stem_chunks) {
  const int bpw = tower16_boards_per_tile(HW, tr);
  if (!bpw) return 0;
  const int nwm = 2, mbw = tr / 16 / nwm;  // blocks per wave
  const double mfma = 16.0 * 16 * 32 * 2;                          // FLOP per v_mfma_f32_16x16x32_f16
  double steps = 0;  // block-k-steps over the tile's waves (4 N quarters per M group)
  for (int h = 0; h < nwm; ++h) {
    int skipped = 0;  // block-taps one wave of this M group skips per conv
    for (int t = 0; t < 9; ++t) skipped += __builtin_popcount((skip[h] >> (2 * t)) & 3);
    // stem: 2 k-steps (4 one-hot planes), or a 36-k-step conv over the input rows (its skips too)
    const double stem = rows_stem ? 9.0 * stem_chunks * mbw - stem_chunks * skipped : 2.0 * mbw;
    const double per_wave = stem + depth * ((4.0 + 36) * mbw + 36.0 * mbw - 2.0 * 4 * skipped);
    steps += 4 * per_wave;
  }
  return steps * 6 * mfma / bpw;  // 2 N blocks x 3 products per block-k-step
}

void tower16_stem_pack(const double* w, int e, std::vector<uint16_t>& out) {
  // conv16_pack's fragment layout ([k-step][n-block][term][lane] x 8 fp16) over k = tap*4 + plane
  const int F = 128;
  out.assign((size_t)2 * 8 * 2 * 64 * 8, 0);
  const double sc = std::ldexp(1.0, -e);
  for (int k = 0; k < 36; ++k)
    for (int co = 0; co < F; ++co) {
      const float ws = (float)(w[(size_t)k * F + co] * sc);  // Keras [3][3][4][F]: k = tap*4 + plane
      const _Float16 b0 = (_Float16)ws;
      const _Float16 b1 = (_Float16)((ws - (float)b0) * 4096.f);
      const _Float16 B0 = (_Float16)((float)b0 * 4096.f);  // exact
      const int ks = k / 32, kk = k % 32, nb = co / 16;
      const int ln = (kk / 8) * 16 + (co % 16), j = kk % 8;
      const size_t base = ((((size_t)ks * 8 + nb) * 2) * 64 + ln) * 8 + j;
      memcpy(&out[base], &B0, 2);
      memcpy(&out[base + 64 * 8], &b1, 2);
    }
}

template <int MBT, int NWM, bool ROWS, bool DB>
static void launch_db(const TowerNet* net, int staged, const Board* boards, const float4* x, const uint4* rows,
                      const int* count, int n_max, int H, int W, int A, float* probs, float* values, float4* feat,
                      int first_chunk, unsigned long long* err, hipStream_t s, TowerLeaves lv = {}) {
  const int bpw = tower16_boards_per_tile(H * W, 16 * MBT);
  const int grid = (n_max + bpw - 1) / bpw;
  const size_t bytes = tower16_lds_bytes(H * W, 16 * MBT, staged, DB);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tower16_kernel<MBT, NWM, ROWS, DB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTowerLdsMax);
    attr = true;
  }
  tower16_kernel<MBT, NWM, ROWS, DB><<<grid, NWM * 256, bytes, s>>>(net, boards, x, rows, count, n_max, H, W, A,
                                                                    bpw, probs, values, feat, first_chunk, err, lv);
}
template <int MBT, int NWM, bool ROWS>
static void launch_mbw(const TowerNet* net, int staged, bool dbuf, const Board* boards, const float4* x,
                       const uint4* rows, const int* count, int n_max, int H, int W, int A, float* probs,
                       float* values, float4* feat, int first_chunk, unsigned long long* err, hipStream_t s,
                       TowerLeaves lv = {}) {
  if (dbuf)
    launch_db<MBT, NWM, ROWS, true>(net, staged, boards, x, rows, count, n_max, H, W, A, probs, values, feat,
                                    first_chunk, err, s, lv);
  else
    launch_db<MBT, NWM, ROWS, false>(net, staged, boards, x, rows, count, n_max, H, W, A, probs, values, feat,
                                     first_chunk, err, s, lv);
}

void launch_tower16(const TowerNet* net, int tile_rows, int alt_rows, int alt_staged, int staged, bool dbuf,
                    const Board* boards,
                    const float4* x, const int* count, int n_max, int H, int W, int A, float* probs, float* values,
                    unsigned long long* err, hipStream_t s) {
  if (n_max <= 0) return;
  if (tile_rows == 128 && alt_rows == 96 && dbuf) {  // Connect-4: 96- or 128-row tiles by the live count
    const int bpw = tower16_boards_per_tile(H * W, 128), bpw2 = tower16_boards_per_tile(H * W, 96);
    const int grid = (n_max + bpw2 - 1) / bpw2;
    const size_t bytes = std::max(tower16_lds_bytes(H * W, 128, staged, true),  // the larger of the two layouts
                                  tower16_lds_bytes(H * W, 96, alt_staged, true));
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tower16_dual_kernel<8, 6, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTowerLdsMax);
      attr = true;
    }
    tower16_dual_kernel<8, 6, true><<<grid, 512, bytes, s>>>(net, boards, x, count, n_max, H, W, A, bpw, bpw2, probs,
                                                             values, err);
    return;
  }
  if (tile_rows == 192)  // in place only (two 192-row tiles exceed the LDS)
    launch_db<12, 2, false, false>(net, staged, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                                   err, s);
  else if (tile_rows == 96)
    launch_mbw<6, 2, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);
  else
    launch_mbw<8, 2, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);
}

void launch_tower16_rows(const TowerNet* net, int tile_rows, int staged, bool dbuf, const void* rows,
                         int first_chunk, const int* count, int n_max, int H, int W, float4* feat,
                         unsigned long long* err, hipStream_t s, const TowerLeaves* leaves) {
  if (n_max <= 0 || tile_rows != 128) return;
  // the leaves' planes are built for the self-play stem (planes 64-127)
  const TowerLeaves lv = leaves && first_chunk == 2 ? *leaves : TowerLeaves{};
  // a launch of fewer than 512 boards (chess self-play: 128 per lane) in
  // 2-board tiles would hold under a quarter of the 256 CUs: one board per
  // 64-row tile then (MI355X has 256 CUs; the same sums, bitwise), 8 waves of
  // 2 blocks.  (16 waves of one block, four per SIMD: 1.16 M against 1.55 M
  // expansions/s, profiles/r5/ab_chess.txt)
  if (n_max < 512)
    launch_mbw<4, 2, true>(net, staged, dbuf, nullptr, nullptr, static_cast<const uint4*>(rows), count, n_max, H, W,
                           0, nullptr, nullptr, feat, first_chunk == 2 ? 2 : 0, err, s, lv);
  else
    launch_mbw<8, 2, true>(net, staged, dbuf, nullptr, nullptr, static_cast<const uint4*>(rows), count, n_max, H, W,
                           0, nullptr, nullptr, feat, first_chunk == 2 ? 2 : 0, err, s, lv);
}

}  // namespace az
