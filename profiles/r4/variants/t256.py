# 256-row in-place tiles (6 C4 boards) on the present 16x16x32 kernel, natural
# order: does halving the weight stream per board pay for the in-place barriers?
# (not run: the in-place kernel spills 424 VGPRs -- two accumulator sets of MBW=6/8 blocks)
s = open("az_tower16.hip").read()
def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)
rep("""  if (HW > 128) return 0;""", """  if (HW > 128) return 0;
  if (HW * 6 <= 256) return 256;""")
rep("const bool planned = 16 * MBT == T.tile_rows;", "const bool planned = MBT <= 8 && 16 * MBT == T.tile_rows;")
rep("""  if (tile_rows == 96)""", """  if (tile_rows == 256)
    launch_db<16, 2, false, false>(net, staged, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                                   err, s);
  else if (tile_rows == 96)""")
open("az_tower16.hip", "w").write(s)
