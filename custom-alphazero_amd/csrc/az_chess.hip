// az_chess.hip -- chess board kernels (encode, legal moves + mask + outcome,
// play, perft) and their C ABI (include/az_chess.h).  The rules live in
// az_chess.h; this file owns the tables, the kernels and the host side.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/az.h"
#include "az_chess.h"

namespace az {
int fail_abi(int code, const std::string& msg);  // az_engine.hip (az_last_error)
}

namespace azc {

namespace {

// get_all_possible_moves() (chess/utils.py:11-32), derived directly: queen
// and knight moves from every square of an empty board, plus the white
// promotions from rank 7 (pushes, and captures onto a full rank 8), each in
// the four promotion pieces; sorted by Move.__lt__ (chess/move.py:33-37):
// (pos_from, pos_to) = ((file, rank), (file, rank, promotion letter)), and
// the letters sort "" < "b" < "n" < "q" < "r".
int promo_rank(int promo) {
  switch (promo) {
    case 0: return 0;
    case BISHOP: return 1;
    case KNIGHT: return 2;
    case QUEEN: return 3;
    default: return 4;
  }
}
int move_key(uint16_t m) {
  int from = m & 63, to = (m >> 6) & 63;
  return ((((from & 7) * 8 + (from >> 3)) * 8 + (to & 7)) * 8 + (to >> 3)) * 5 + promo_rank(m >> 12);
}
const std::vector<uint16_t>& all_moves() {
  static std::vector<uint16_t> mv;
  static std::once_flag once;
  std::call_once(once, [] {
    uint64_t rays[8][64];
    host_rays(rays);
    static const int kn[8][2] = {{1, 2}, {2, 1}, {2, -1}, {1, -2}, {-1, -2}, {-2, -1}, {-2, 1}, {-1, 2}};
    for (int s = 0; s < 64; ++s) {
      for (int d = 0; d < 8; ++d)
        for (uint64_t r = rays[d][s]; r; r &= r - 1) mv.push_back((uint16_t)(s | (__builtin_ctzll(r) << 6)));
      for (int i = 0; i < 8; ++i) {
        int f = (s & 7) + kn[i][0], k = (s >> 3) + kn[i][1];
        if (f >= 0 && f < 8 && k >= 0 && k < 8) mv.push_back((uint16_t)(s | ((k * 8 + f) << 6)));
      }
    }
    for (int f = 0; f < 8; ++f)
      for (int df = -1; df <= 1; ++df) {
        if (f + df < 0 || f + df > 7) continue;
        for (int promo = KNIGHT; promo <= QUEEN; ++promo)
          mv.push_back((uint16_t)((48 + f) | ((56 + f + df) << 6) | (promo << 12)));
      }
    std::sort(mv.begin(), mv.end(), [](uint16_t a, uint16_t b) { return move_key(a) < move_key(b); });
    mv.erase(std::unique(mv.begin(), mv.end()), mv.end());
  });
  return mv;
}

}  // namespace

// move -> action index table [from][to][promo slot], -1 = not an action
std::vector<int16_t> action_lut() {
  std::vector<int16_t> lut(64 * 64 * 5, -1);
  const auto& mv = all_moves();
  for (size_t i = 0; i < mv.size(); ++i) {
    uint16_t m = mv[i];
    int promo = m >> 12;
    lut[((m & 63) * 64 + ((m >> 6) & 63)) * 5 + (promo ? promo - 1 : 0)] = (int16_t)i;
  }
  return lut;
}

namespace {

// per-device state: stream, tables, action table
struct DevCtx {
  bool ready = false;
  hipStream_t stream = nullptr;
  int16_t* lut = nullptr;
};
std::mutex g_mu;
DevCtx g_ctx[64];

#define AZC_HIP(expr)                                                                          \
  do {                                                                                         \
    hipError_t err__ = (expr);                                                                 \
    if (err__ != hipSuccess)                                                                   \
      return az::fail_abi(AZ_E_HIP, std::string(#expr) + ": " + hipGetErrorString(err__));     \
  } while (0)

int ctx_for(int device, DevCtx** out) {
  if (device < 0 || device >= 64) return az::fail_abi(AZ_E_INVALID, "chess: bad device ordinal");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
    return az::fail_abi(AZ_E_HIP, "chess: no HIP device visible (libaz has no CPU fallback)");
  if (device >= count) return az::fail_abi(AZ_E_INVALID, "chess: device ordinal out of range");
  AZC_HIP(hipSetDevice(device));
  std::lock_guard<std::mutex> lk(g_mu);
  DevCtx& c = g_ctx[device];
  if (!c.ready) {
    AZC_HIP(upload_rays());
    AZC_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    std::vector<int16_t> lut = action_lut();
    AZC_HIP(hipMalloc(&c.lut, lut.size() * sizeof(int16_t)));
    AZC_HIP(hipMemcpy(c.lut, lut.data(), lut.size() * sizeof(int16_t), hipMemcpyHostToDevice));
    c.ready = true;
  }
  *out = &c;
  return AZ_OK;
}

// device buffer that frees itself
template <class T>
struct DBuf {
  T* p = nullptr;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t n) { return hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)); }
};

}  // namespace

// ----------------------------------------------------------------- kernels

// Board.moves / legal_moves_mask / outcome, one thread per position.  The
// move list is generated straight into the position's output row (pseudo-
// legal first, then compacted in place by the _is_safe filter).
__global__ void __launch_bounds__(64) legal_kernel(const az_chess_pos* __restrict__ pos, int n,
                                                   uint16_t* __restrict__ moves, int32_t* counts,
                                                   uint8_t* __restrict__ mask, int32_t* outcome_out,
                                                   const int16_t* __restrict__ lut) {
  // one wave per position with the self-play leaves' generator
  // (legal_moves_wave), so the Board API and its tests exercise it; the
  // perft kernels keep the one-thread legal_moves: both are pinned
  __shared__ uint16_t cand[AZ_CHESS_MAX_MOVES];
  const int i = blockIdx.x, lane = threadIdx.x;
  if (i >= n) return;
  const Pos q = load_pos(pos[i]);
  uint16_t* row = moves + (size_t)i * AZ_CHESS_MAX_MOVES;
  bool check;
  const int k = legal_moves_wave(q, cand, row, &check, lane);
  if (lane == 0) counts[i] = k;
  if (k < 0) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (mask) {
    uint8_t* mrow = mask + (size_t)i * AZ_CHESS_ACTIONS;
    for (int j = lane; j < k; j += 64) {
      const int a = action_of(lut, row[j]);
      if (a >= 0) mrow[a] = 1;
    }
  }
  if (outcome_out && lane == 0) outcome_out[i] = outcome(q, k, check);
}

// Board.full_state for n boards: one workgroup per board, its 8 history
// positions in LDS; consecutive threads write consecutive floats of the
// [8][8][118] NHWC state (coalesced).
__global__ void __launch_bounds__(256) encode_kernel(const az_chess_pos* __restrict__ hist,
                                                     const uint8_t* __restrict__ valid, int n,
                                                     float* __restrict__ out) {
  __shared__ Pos sp[AZ_CHESS_HISTORY];
  __shared__ int sv[AZ_CHESS_HISTORY];
  __shared__ float feat[6];
  for (int b = blockIdx.x; b < n; b += gridDim.x) {
    __syncthreads();
    if (threadIdx.x < AZ_CHESS_HISTORY) {
      sp[threadIdx.x] = load_pos(hist[(size_t)b * AZ_CHESS_HISTORY + threadIdx.x]);
      sv[threadIdx.x] = valid[(size_t)b * AZ_CHESS_HISTORY + threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const Pos& cur = sp[AZ_CHESS_HISTORY - 1];
      bb c = clean_castling(cur);
      bb back_t = cur.turn ? RANK_1 : RANK_8, back_o = cur.turn ? RANK_8 : RANK_1;
      feat[0] = (c & FILE_A & back_t) != 0;  // has_queenside_castling_rights(turn)
      feat[1] = (c & FILE_H & back_t) != 0;  // has_kingside_castling_rights(turn)
      feat[2] = (c & FILE_A & back_o) != 0;
      feat[3] = (c & FILE_H & back_o) != 0;
      feat[4] = (float)cur.full;
      feat[5] = (float)cur.half;
    }
    __syncthreads();
    float* o = out + (size_t)b * 64 * AZ_CHESS_PLANES;
    for (int e = threadIdx.x; e < 64 * AZ_CHESS_PLANES; e += blockDim.x) {
      int pix = e / AZ_CHESS_PLANES, k = e - pix * AZ_CHESS_PLANES;
      int sq = (7 - (pix >> 3)) * 8 + (pix & 7);  // row 0 = rank 8 (Board.array)
      float v;
      if (k >= 112) {
        v = feat[k - 112];
      } else {
        int h = k / 14, j = k - h * 14;
        if (!sv[h]) v = 0.f;
        else if (j == 13) v = (float)sp[h].rep;
        else v = onehot_index(sp[h], sq) == j ? 1.f : 0.f;
      }
      o[e] = v;
    }
  }
}

__global__ void play_kernel(az_chess_pos* pos, const uint16_t* __restrict__ moves, int n, int keep) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Pos q = load_pos(pos[i]);
  play(q, moves[i], keep != 0);
  store_pos(q, pos[i]);
}

// perft: the legal moves of every position of a level into a global move
// table [n][AZ_CHESS_MAX_MOVES] (no per-lane scratch array), their counts and
// sum
__global__ void __launch_bounds__(128) perft_count_kernel(const az_chess_pos* __restrict__ pos, int n,
                                                          uint16_t* __restrict__ moves, int32_t* counts,
                                                          unsigned long long* total, int* err) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  int k = 0;
  if (i < n) {
    bool check;
    Pos q = load_pos(pos[i]);
    k = legal_moves(q, moves + (size_t)i * AZ_CHESS_MAX_MOVES, &check);
    if (k < 0) {
      atomicOr(err, 1);
      k = 0;
    }
    counts[i] = k;
  }
  // wave-level sum before the one atomic per wave
  unsigned long long s = (unsigned long long)k;
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(total, s);
}

// perft: expand a level into the next (children at the exclusive-scan offsets)
__global__ void __launch_bounds__(128) perft_expand_kernel(const az_chess_pos* __restrict__ pos, int n,
                                                           const uint16_t* __restrict__ moves,
                                                           const int32_t* __restrict__ counts,
                                                           const long long* __restrict__ offs,
                                                           az_chess_pos* __restrict__ next) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Pos q = load_pos(pos[i]);
  const int k = counts[i];
  const long long o = offs[i];
  for (int j = 0; j < k; ++j) {
    Pos c = q;
    push(c, moves[(size_t)i * AZ_CHESS_MAX_MOVES + j]);
    store_pos(c, next[o + j]);
  }
}

}  // namespace azc

// -------------------------------------------------------------------- ABI
using namespace azc;

extern "C" int az_chess_all_moves(uint16_t* out, int cap) {
  const auto& mv = all_moves();
  if (!out || cap < (int)mv.size()) return az::fail_abi(AZ_E_INVALID, "az_chess_all_moves: cap too small");
  memcpy(out, mv.data(), mv.size() * sizeof(uint16_t));
  return (int)mv.size();
}

extern "C" int az_chess_legal(int device, const az_chess_pos* pos, int n, uint16_t* moves,
                              int32_t* counts, uint8_t* mask, int32_t* outcome_out) {
  if (n < 0 || (n > 0 && (!pos || !counts))) return az::fail_abi(AZ_E_INVALID, "az_chess_legal: bad arguments");
  if (n == 0) return AZ_OK;
  DevCtx* c;
  if (int rc = ctx_for(device, &c)) return rc;
  DBuf<az_chess_pos> dpos;
  DBuf<uint16_t> dmv;
  DBuf<int32_t> dcnt, dout;
  DBuf<uint8_t> dmask;
  AZC_HIP(dpos.alloc(n));
  AZC_HIP(dmv.alloc((size_t)n * AZ_CHESS_MAX_MOVES));
  AZC_HIP(dcnt.alloc(n));
  if (outcome_out) AZC_HIP(dout.alloc(n));
  if (mask) {
    AZC_HIP(dmask.alloc((size_t)n * AZ_CHESS_ACTIONS));
    AZC_HIP(hipMemsetAsync(dmask.p, 0, (size_t)n * AZ_CHESS_ACTIONS, c->stream));
  }
  AZC_HIP(hipMemcpyAsync(dpos.p, pos, sizeof(az_chess_pos) * n, hipMemcpyHostToDevice, c->stream));
  legal_kernel<<<n, 64, 0, c->stream>>>(dpos.p, n, dmv.p, dcnt.p, mask ? dmask.p : nullptr,
                                                      outcome_out ? dout.p : nullptr, c->lut);
  AZC_HIP(hipGetLastError());
  AZC_HIP(hipMemcpyAsync(counts, dcnt.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  if (moves)
    AZC_HIP(hipMemcpyAsync(moves, dmv.p, sizeof(uint16_t) * AZ_CHESS_MAX_MOVES * n, hipMemcpyDeviceToHost,
                           c->stream));
  if (mask)
    AZC_HIP(hipMemcpyAsync(mask, dmask.p, (size_t)n * AZ_CHESS_ACTIONS, hipMemcpyDeviceToHost, c->stream));
  if (outcome_out)
    AZC_HIP(hipMemcpyAsync(outcome_out, dout.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  AZC_HIP(hipStreamSynchronize(c->stream));
  for (int i = 0; i < n; ++i)
    if (counts[i] < 0) return az::fail_abi(AZ_E_DEVICE, "az_chess_legal: pseudo-legal move list overflow");
  return AZ_OK;
}

extern "C" int az_chess_encode(int device, const az_chess_pos* hist, const uint8_t* valid, int n,
                               float* state) {
  if (n < 0 || (n > 0 && (!hist || !valid || !state)))
    return az::fail_abi(AZ_E_INVALID, "az_chess_encode: bad arguments");
  if (n == 0) return AZ_OK;
  DevCtx* c;
  if (int rc = ctx_for(device, &c)) return rc;
  DBuf<az_chess_pos> dh;
  DBuf<uint8_t> dv;
  DBuf<float> ds;
  size_t per = (size_t)64 * AZ_CHESS_PLANES;
  AZC_HIP(dh.alloc((size_t)n * AZ_CHESS_HISTORY));
  AZC_HIP(dv.alloc((size_t)n * AZ_CHESS_HISTORY));
  AZC_HIP(ds.alloc((size_t)n * per));
  AZC_HIP(hipMemcpyAsync(dh.p, hist, sizeof(az_chess_pos) * AZ_CHESS_HISTORY * n, hipMemcpyHostToDevice,
                         c->stream));
  AZC_HIP(hipMemcpyAsync(dv.p, valid, (size_t)AZ_CHESS_HISTORY * n, hipMemcpyHostToDevice, c->stream));
  encode_kernel<<<std::min(n, 4096), 256, 0, c->stream>>>(dh.p, dv.p, n, ds.p);
  AZC_HIP(hipGetLastError());
  AZC_HIP(hipMemcpyAsync(state, ds.p, sizeof(float) * per * n, hipMemcpyDeviceToHost, c->stream));
  AZC_HIP(hipStreamSynchronize(c->stream));
  return AZ_OK;
}

extern "C" int az_chess_play(int device, az_chess_pos* pos, const uint16_t* moves, int n, int keep_same_player) {
  if (n < 0 || (n > 0 && (!pos || !moves))) return az::fail_abi(AZ_E_INVALID, "az_chess_play: bad arguments");
  if (n == 0) return AZ_OK;
  DevCtx* c;
  if (int rc = ctx_for(device, &c)) return rc;
  DBuf<az_chess_pos> dp;
  DBuf<uint16_t> dm;
  AZC_HIP(dp.alloc(n));
  AZC_HIP(dm.alloc(n));
  AZC_HIP(hipMemcpyAsync(dp.p, pos, sizeof(az_chess_pos) * n, hipMemcpyHostToDevice, c->stream));
  AZC_HIP(hipMemcpyAsync(dm.p, moves, sizeof(uint16_t) * n, hipMemcpyHostToDevice, c->stream));
  play_kernel<<<(n + 127) / 128, 128, 0, c->stream>>>(dp.p, dm.p, n, keep_same_player);
  AZC_HIP(hipGetLastError());
  AZC_HIP(hipMemcpyAsync(pos, dp.p, sizeof(az_chess_pos) * n, hipMemcpyDeviceToHost, c->stream));
  AZC_HIP(hipStreamSynchronize(c->stream));
  return AZ_OK;
}

extern "C" int az_chess_perft(int device, const az_chess_pos* pos, int depth, uint64_t* nodes) {
  if (!pos || !nodes || depth < 0 || depth > 8) return az::fail_abi(AZ_E_INVALID, "az_chess_perft: bad arguments");
  if (depth == 0) {
    *nodes = 1;
    return AZ_OK;
  }
  DevCtx* c;
  if (int rc = ctx_for(device, &c)) return rc;
  DBuf<az_chess_pos> level;
  AZC_HIP(level.alloc(1));
  AZC_HIP(hipMemcpyAsync(level.p, pos, sizeof(az_chess_pos), hipMemcpyHostToDevice, c->stream));
  long long n = 1;
  DBuf<unsigned long long> dtot;
  DBuf<int> derr;
  AZC_HIP(dtot.alloc(1));
  AZC_HIP(derr.alloc(1));
  AZC_HIP(hipMemsetAsync(derr.p, 0, sizeof(int), c->stream));
  const long long kMaxLevel = 1ll << 26;  // 5.4 GB of positions (+ 34 GB of move lists)
  for (int d = 1; d <= depth; ++d) {
    DBuf<int32_t> cnt;
    DBuf<uint16_t> mv;
    AZC_HIP(cnt.alloc(n));
    AZC_HIP(mv.alloc((size_t)n * AZ_CHESS_MAX_MOVES));
    AZC_HIP(hipMemsetAsync(dtot.p, 0, sizeof(unsigned long long), c->stream));
    int blocks = (int)((n + 127) / 128);
    perft_count_kernel<<<blocks, 128, 0, c->stream>>>(level.p, (int)n, mv.p, cnt.p, dtot.p, derr.p);
    AZC_HIP(hipGetLastError());
    unsigned long long tot = 0;
    int err = 0;
    AZC_HIP(hipMemcpyAsync(&tot, dtot.p, sizeof(tot), hipMemcpyDeviceToHost, c->stream));
    AZC_HIP(hipMemcpyAsync(&err, derr.p, sizeof(err), hipMemcpyDeviceToHost, c->stream));
    AZC_HIP(hipStreamSynchronize(c->stream));
    if (err) return az::fail_abi(AZ_E_DEVICE, "az_chess_perft: pseudo-legal move list overflow");
    if (d == depth) {
      *nodes = tot;
      return AZ_OK;
    }
    if ((long long)tot > kMaxLevel) return az::fail_abi(AZ_E_INVALID, "az_chess_perft: level too large");
    // exclusive scan of the counts on the host (a test utility, not a hot path)
    std::vector<int32_t> hc(n);
    std::vector<long long> ho(n);
    AZC_HIP(hipMemcpy(hc.data(), cnt.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    long long run = 0;
    for (long long i = 0; i < n; ++i) {
      ho[i] = run;
      run += hc[i];
    }
    DBuf<long long> doff;
    DBuf<az_chess_pos> next;
    AZC_HIP(doff.alloc(n));
    AZC_HIP(next.alloc(run));
    AZC_HIP(hipMemcpy(doff.p, ho.data(), sizeof(long long) * n, hipMemcpyHostToDevice));
    perft_expand_kernel<<<blocks, 128, 0, c->stream>>>(level.p, (int)n, mv.p, cnt.p, doff.p, next.p);
    AZC_HIP(hipGetLastError());
    AZC_HIP(hipStreamSynchronize(c->stream));
    std::swap(level.p, next.p);
    n = run;
  }
  return AZ_OK;
}
