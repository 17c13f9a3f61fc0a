# 192-row in-place tiles (4 C4 boards, 2 9x9 boards) on the present kernel,
# natural order: the weight stream amortised over twice the pixels
# (round 5: on the assembly K loop; round 4 spilled 163 VGPRs)
s = open("az_tower16.hip").read()
def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)
rep("""  if (HW > 128) return 0;""", """  if (HW > 128) return 0;
  if (HW * 2 <= 192 && HW > 42) return 192;
  if (HW == 42) return 192;""")
rep("const bool planned = 16 * MBT == T.tile_rows;", "const bool planned = MBT <= 8 && 16 * MBT == T.tile_rows;")
rep("""  if (tile_rows == 96)""", """  if (tile_rows == 192)
    launch_db<12, 2, false, false>(net, staged, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                                   err, s);
  else if (tile_rows == 96)""")
open("az_tower16.hip", "w").write(s)
