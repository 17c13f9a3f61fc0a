// Host build of the device chess rules (csrc/az_chess.h) under AddressSanitizer
// + UBSan, checked against the oracle (oracle/chess_oracle.c) over the perft
// trees of the standard positions (tests/test_chess_oracle.py).  TEST
// INFRASTRUCTURE (tests/test_chess_native_cpu.py builds and runs it).
//
// At every interior node: legal_moves twice (the count pass and the expand
// pass of the round-1 device perft, which once disagreed run to run) must give
// the same list, equal to the oracle's, and the leaf counts must be the
// published perft numbers.  At every 61st node (and the roots) the network
// input planes the chess tower builds from a queued leaf (az_chess.h
// state_feats / full_state4, planes 64-127, both history forms) must equal
// the oracle's Board.full_state (orc_chess_full_state), planes 0-63 zero.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../custom-alphazero_amd/csrc/az_chess.h"

extern "C" {
int orc_chess_from_fen(const char* fen, az_chess_pos* out);
int orc_chess_legal(const az_chess_pos* p, uint16_t* out);
void orc_chess_push(az_chess_pos* p, uint16_t m);
void orc_chess_full_state(const az_chess_pos* hist, const uint8_t* valid, const az_chess_pos* cur, double* out);
}

static long long g_nodes = 0, g_fail = 0, g_planes = 0;

// full_state4 against the oracle for position cp as a played board (history
// [0 x 6, start, cp]) and as a reset root ([0 x 7, start-position state])
static void planes_check(const az_chess_pos& cp) {
  az_chess_pos start;
  orc_chess_from_fen("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", &start);
  std::vector<double> ref(64 * 118);
  const azc::Pos st = azc::start_pos(), cur = azc::load_pos(cp);
  float f[6];
  azc::state_feats(cur, f);
  for (int initial = 0; initial < 2; ++initial) {
    az_chess_pos hist[8];
    uint8_t valid[8] = {0, 0, 0, 0, 0, 0, 0, 1};
    for (auto& h : hist) h = start;
    if (!initial) {
      hist[7] = cp;
      valid[6] = 1;
    }
    orc_chess_full_state(hist, valid, &cp, ref.data());
    long bad = 0;
    for (int pix = 0; pix < 64; ++pix) {
      for (int k = 0; k < 64; ++k) bad += ref[pix * 118 + k] != 0.0;
      for (int k0 = 64; k0 < 128; k0 += 4) {
        float v[4];
        azc::full_state4(st, cur, initial != 0, f, pix, k0, v);
        for (int i = 0; i < 4; ++i) {
          const int k = k0 + i;
          bad += (double)v[i] != (k < 118 ? ref[pix * 118 + k] : 0.0);
        }
      }
    }
    ++g_planes;
    if (bad && g_fail++ < 5) fprintf(stderr, "planes mismatch (%ld, initial %d)\n", bad, initial);
  }
}

static unsigned long long walk(const azc::Pos& q, int depth) {
  // move buffers sized exactly AZ_CHESS_MAX_MOVES: ASan sees any write past them
  std::vector<uint16_t> a(AZ_CHESS_MAX_MOVES), b(AZ_CHESS_MAX_MOVES), o(256);
  bool ca = false, cb = false;
  const int na = azc::legal_moves(q, a.data(), &ca);
  const int nb = azc::legal_moves(q, b.data(), &cb);
  az_chess_pos cp;
  azc::store_pos(q, cp);
  const int no = orc_chess_legal(&cp, o.data());
  if (g_nodes % 61 == 0) planes_check(cp);
  ++g_nodes;
  if (na != nb || ca != cb || na != no || memcmp(a.data(), b.data(), na * 2) || memcmp(a.data(), o.data(), na * 2)) {
    if (g_fail++ < 5) fprintf(stderr, "mismatch: %d/%d vs oracle %d\n", na, nb, no);
    return 0;
  }
  if (depth == 1) return (unsigned long long)na;
  unsigned long long s = 0;
  for (int i = 0; i < na; ++i) {
    azc::Pos c = q;
    azc::push(c, a[i]);
    // the oracle's push of the same move must give the same position
    az_chess_pos po = cp, pd;
    orc_chess_push(&po, a[i]);
    azc::store_pos(c, pd);
    if (memcmp(&po, &pd, sizeof(po))) {
      if (g_fail++ < 5) fprintf(stderr, "push mismatch\n");
      continue;
    }
    s += walk(c, depth - 1);
  }
  return s;
}

int main() {
  struct Case {
    const char* fen;
    std::vector<unsigned long long> counts;
  } cases[] = {
      {"rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", {20, 400, 8902, 197281, 4865609}},
      {"r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", {48, 2039, 97862, 4085603}},
      {"8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1", {14, 191, 2812, 43238, 674624}},
      {"r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1", {6, 264, 9467, 422333}},
      {"rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8", {44, 1486, 62379, 2103487}},
      {"r4rk1/1pp1qppp/p1np1n2/2b1p1B1/2B1P1b1/P1NP1N2/1PP1QPPP/R4RK1 w - - 0 10", {46, 2079, 89890, 3894594}},
  };
  int bad = 0;
  for (const Case& c : cases) {
    az_chess_pos p;
    if (orc_chess_from_fen(c.fen, &p)) {
      fprintf(stderr, "bad fen %s\n", c.fen);
      return 2;
    }
    const int d = (int)c.counts.size();
    const unsigned long long got = walk(azc::load_pos(p), d);
    printf("perft(%d) %llu (expected %llu) %s\n", d, got, c.counts[d - 1], c.fen);
    bad += got != c.counts[d - 1];
  }
  printf("nodes generated %lld, input planes checked %lld, mismatches %lld\n", g_nodes, g_planes, g_fail);
  return bad || g_fail ? 1 : 0;
}
