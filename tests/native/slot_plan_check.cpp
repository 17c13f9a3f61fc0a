// Checks the tower's slot plan (az::tower16_slot_plan, libaz.so host code)
// over board shapes: every pixel of a full tile in exactly one slot, every
// skipped (block, tap) pair adding exact zeros (each pixel of the block has
// its tap neighbour off the board), and the LDS bank residues of each
// ds_read_b128 lane group.  One JSON object per shape on stdout.
#include <cstdio>
#include <vector>

namespace az {
void tower16_slot_plan(int H, int W, int tile_rows, std::vector<int>& slot_pix, int skip[2]);
int tower16_tile_rows(int HW);
int tower16_boards_per_tile(int HW, int tile_rows);
}  // namespace az

int main() {
  const int S1[8] = {0, 1, 2, 3, 12, 13, 14, 15}, S2[8] = {4, 5, 6, 7, 8, 9, 10, 11};
  bool first = true;
  printf("[");
  for (int H = 3; H <= 11; ++H)
    for (int W = 3; W <= 11; ++W)
      for (int alt = 0; alt < 2; ++alt) {
      // alt: the dual launch's 96-row tiles of two boards beside 128-row tiles
      // of three (round 6, Connect-4's shape class)
      const int HW = H * W, tr0 = az::tower16_tile_rows(HW);
      const bool dual = tr0 == 128 && az::tower16_boards_per_tile(HW, 128) == 3 &&
                        az::tower16_boards_per_tile(HW, 96) == 2;
      if (!tr0 || (alt && !dual)) continue;
      const int tr = alt ? 96 : tr0;
      const int nb = az::tower16_boards_per_tile(HW, tr), half = tr / 32;
      std::vector<int> pix;
      int skip[2];
      az::tower16_slot_plan(H, W, tr, pix, skip);
      int dup = 0, missing = 0, bad_skip = 0, pads = 0, conflicts = 0, skipped = 0;
      if (!pix.empty()) {
        std::vector<int> seen(nb * HW, 0);
        for (int v : pix) {
          const int y = (v >> 8) & 255, x = v & 255, b = v >> 16;
          if (y == 127) {
            ++pads;
            continue;
          }
          if (b >= nb || y >= H || x >= W) {
            ++bad_skip;
            continue;
          }
          if (seen[b * HW + y * W + x]++) ++dup;
        }
        for (int c : seen) missing += c == 0;
        for (int h = 0; h < 2; ++h)
          for (int t = 0; t < 9; ++t)
            for (int bit = 0; bit < 2; ++bit) {
              if (!((skip[h] >> (2 * t + bit)) & 1)) continue;
              ++skipped;
              const int blk = h * half + bit, dy = t / 3 - 1, dx = t % 3 - 1;
              for (int j = 0; j < 16; ++j) {
                const int v = pix[blk * 16 + j], y = (v >> 8) & 255, x = v & 255;
                if (y == 127) continue;
                if (y + dy >= 0 && y + dy < H && x + dx >= 0 && x + dx < W) ++bad_skip;
              }
            }
        for (int blk = 0; blk < tr / 16; ++blk)
          for (const int* S : {S1, S2}) {
            int cnt[8] = {0};
            for (int i = 0; i < 8; ++i) {
              const int v = pix[blk * 16 + S[i]], y = (v >> 8) & 255, x = v & 255, b = v >> 16;
              const int row = y == 127 ? x : b * HW + y * W + x;
              ++cnt[row & 7];
            }
            for (int r = 0; r < 8; ++r) conflicts += cnt[r] > 1 ? cnt[r] - 1 : 0;
          }
      }
      printf("%s{\"H\": %d, \"W\": %d, \"tile_rows\": %d, \"alt\": %d, \"boards\": %d, \"plan\": %d, \"dup\": %d, "
             "\"missing\": %d, \"bad\": %d, \"pads\": %d, \"skipped_block_taps\": %d, \"conflicts\": %d}",
             first ? "" : ",\n", H, W, tr, alt, nb, (int)!pix.empty(), dup, missing, bad_skip, pads, skipped, conflicts);
      first = false;
    }
  printf("]\n");
  return 0;
}
