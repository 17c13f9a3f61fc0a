// Reconstruction of the round-1 device perft whose Kiwipete depth-4 count
// varied run to run (DESIGN.md "Scratch memory"), to find the cause.  TEST
// INFRASTRUCTURE, run on the GPU by tests/test_chess_gpu.py.
//
// Round-1 scheme: a count kernel and an expand kernel each generate a
// position's legal moves into a per-lane array (scratch), the host scans the
// counts into child offsets and uploads them with a synchronous hipMemcpy,
// then the expand kernel -- on a NON-BLOCKING stream -- pushes the children
// at those offsets.  Modes:
//   0  that scheme as it was (offsets: hipMemcpy on the null stream)
//   1  offsets by hipMemcpyAsync on the kernel's own stream
// Each mode records both passes' move lists and reports positions where they
// differ, and the perft totals over several repetitions.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../custom-alphazero_amd/csrc/az_chess.h"

using namespace azc;

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(3);                                                               \
    }                                                                        \
  } while (0)

__global__ void __launch_bounds__(128) count_kernel(const az_chess_pos* pos, int n, int32_t* counts,
                                                    uint16_t* list_a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint16_t buf[AZ_CHESS_MAX_MOVES];  // per-lane array: scratch, as in round 1
  bool check;
  const Pos q = load_pos(pos[i]);
  const int k = legal_moves(q, buf, &check);
  counts[i] = k;
  for (int j = 0; j < k; ++j) list_a[(size_t)i * AZ_CHESS_MAX_MOVES + j] = buf[j];
}

__global__ void __launch_bounds__(128) expand_kernel(const az_chess_pos* pos, int n, const long long* offs,
                                                     az_chess_pos* next, uint16_t* list_b, int32_t* counts_b) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint16_t buf[AZ_CHESS_MAX_MOVES];
  bool check;
  const Pos q = load_pos(pos[i]);
  const int k = legal_moves(q, buf, &check);
  counts_b[i] = k;
  const long long o = offs[i];
  for (int j = 0; j < k; ++j) {
    list_b[(size_t)i * AZ_CHESS_MAX_MOVES + j] = buf[j];
    Pos c = q;
    push(c, buf[j]);
    store_pos(c, next[o + j]);
  }
}

extern "C" int orc_chess_from_fen(const char* fen, az_chess_pos* out);

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int depth = 4;
  const unsigned long long expected = 4085603;  // Kiwipete perft(4)
  az_chess_pos root;
  if (orc_chess_from_fen("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", &root)) return 2;
  CK(upload_rays());
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int bad_runs = 0;
  long long list_mismatch = 0, count_mismatch = 0;
  for (int rep = 0; rep < reps; ++rep) {
    az_chess_pos* level;
    CK(hipMalloc(&level, sizeof(az_chess_pos)));
    CK(hipMemcpy(level, &root, sizeof(root), hipMemcpyHostToDevice));
    long long n = 1;
    unsigned long long total = 0;
    for (int d = 1; d <= depth; ++d) {
      int32_t *cnt, *cnt_b;
      uint16_t *la, *lb;
      CK(hipMalloc(&cnt, n * 4));
      CK(hipMalloc(&cnt_b, n * 4));
      CK(hipMalloc(&la, n * AZ_CHESS_MAX_MOVES * 2));
      CK(hipMalloc(&lb, n * AZ_CHESS_MAX_MOVES * 2));
      const int blocks = (int)((n + 127) / 128);
      count_kernel<<<blocks, 128, 0, st>>>(level, (int)n, cnt, la);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(st));
      std::vector<int32_t> hc(n);
      CK(hipMemcpy(hc.data(), cnt, n * 4, hipMemcpyDeviceToHost));
      std::vector<long long> ho(n);
      long long run = 0;
      for (long long i = 0; i < n; ++i) {
        ho[i] = run;
        run += hc[i];
      }
      if (d == depth) {
        total = (unsigned long long)run;
        CK(hipFree(cnt));
        CK(hipFree(cnt_b));
        CK(hipFree(la));
        CK(hipFree(lb));
        break;
      }
      long long* doff;
      az_chess_pos* next;
      CK(hipMalloc(&doff, n * 8));
      CK(hipMalloc(&next, run * sizeof(az_chess_pos)));
      if (mode == 0) {
        CK(hipMemcpy(doff, ho.data(), n * 8, hipMemcpyHostToDevice));
      } else {
        CK(hipMemcpyAsync(doff, ho.data(), n * 8, hipMemcpyHostToDevice, st));
      }
      expand_kernel<<<blocks, 128, 0, st>>>(level, (int)n, doff, next, lb, cnt_b);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(st));
      // both passes' lists
      std::vector<int32_t> hb(n);
      std::vector<uint16_t> ha((size_t)n * AZ_CHESS_MAX_MOVES), hbl((size_t)n * AZ_CHESS_MAX_MOVES);
      CK(hipMemcpy(hb.data(), cnt_b, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(ha.data(), la, ha.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hbl.data(), lb, hbl.size() * 2, hipMemcpyDeviceToHost));
      for (long long i = 0; i < n; ++i) {
        if (hb[i] != hc[i]) {
          ++count_mismatch;
          continue;
        }
        for (int j = 0; j < hc[i]; ++j)
          if (ha[(size_t)i * AZ_CHESS_MAX_MOVES + j] != hbl[(size_t)i * AZ_CHESS_MAX_MOVES + j]) {
            ++list_mismatch;
            break;
          }
      }
      CK(hipFree(cnt));
      CK(hipFree(cnt_b));
      CK(hipFree(la));
      CK(hipFree(lb));
      CK(hipFree(doff));
      CK(hipFree(level));
      level = next;
      n = run;
    }
    CK(hipFree(level));
    printf("mode %d rep %d: perft(%d) %llu (expected %llu)\n", mode, rep, depth, total, expected);
    bad_runs += total != expected;
  }
  printf("mode %d: %d of %d runs wrong, %lld count mismatches, %lld list mismatches between the passes\n", mode,
         bad_runs, reps, count_mismatch, list_mismatch);
  return bad_runs || count_mismatch || list_mismatch ? 1 : 0;
}
