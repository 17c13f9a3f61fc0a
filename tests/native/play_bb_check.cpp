// Host check of the bitboard Board.play (play_bb, az_device.h) against the
// cell-scan play(): every action from every position of random games, over
// Connect-N configurations with and without gravity (tests/test_board_cpu.py).
#include <cstdio>
#include <cstring>
#include <random>

#include "az_device.h"

int main() {
  struct Cfg { int H, W, n, gravity; };
  const Cfg cfgs[] = {{6, 7, 4, 1}, {4, 4, 3, 1}, {5, 5, 4, 0}, {3, 3, 3, 0}, {9, 9, 5, 1}, {8, 1, 4, 1},
                      {1, 8, 4, 1}, {6, 7, 5, 1}, {2, 64, 4, 1}, {11, 11, 5, 0}, {4, 5, 6, 1}, {8, 16, 4, 0},
                      {16, 8, 9, 1}, {7, 6, 4, 0}};
  std::mt19937_64 rng(12345);
  long checked = 0, checked_c64 = 0, bad = 0;
  for (const Cfg& cf : cfgs) {
    az::GameCfg g{};
    g.H = cf.H; g.W = cf.W; g.HW = cf.H * cf.W; g.n = cf.n; g.gravity = cf.gravity;
    g.A = cf.gravity ? cf.W : g.HW;
    const az::BoardMasks mk = az::board_masks(g);
    for (int game = 0; game < 300; ++game) {
      az::Board b{};
      for (int ply = 0; ply <= g.HW; ++ply) {
        for (int a = 0; a < g.A; ++a) {
          az::Board b1 = b, b2 = b;
          const int s1 = az::play(g, b1, a), s2 = az::play_bb(g, mk, b2, a);
          ++checked;
          if (s1 != s2 || (s1 >= 0 && memcmp(&b1, &b2, sizeof(b1)) != 0)) {
            if (++bad < 10) printf("mismatch H=%d W=%d n=%d grav=%d ply=%d a=%d: %d vs %d\n", g.H, g.W, g.n,
                                   g.gravity, ply, a, s1, s2);
          }
          // the compile-time one-word form the select descent uses for Connect-4
          if (cf.H == 6 && cf.W == 7 && cf.n == 4 && cf.gravity) {
            az::Board b3 = b;
            const int s3 = az::play_c64<6, 7, 4>(b3, a);
            ++checked_c64;
            if (s1 != s3 || (s1 >= 0 && memcmp(&b1, &b3, sizeof(b1)) != 0)) {
              if (++bad < 10) printf("play_c64 mismatch ply=%d a=%d: %d vs %d\n", ply, a, s1, s3);
            }
          }
        }
        int legal[az::kMaxActions], nl = 0;
        for (int a = 0; a < g.A; ++a) {
          az::Board t = b;
          if (az::play(g, t, a) >= 0) legal[nl++] = a;
        }
        if (nl == 0) break;
        const int st = az::play(g, b, legal[rng() % nl]);
        if (st != az::kOngoing) break;
      }
    }
  }
  printf("play_bb: %ld actions checked (%ld also by play_c64<6,7,4>), %ld mismatches\n", checked, checked_c64, bad);
  return bad ? 1 : 0;
}
