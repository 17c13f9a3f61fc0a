# The dual launch's 96-row tiles in 4 waves (one per SIMD, all 6 M blocks
# per wave: NWM = 1) instead of 8 (two M halves of 3 blocks): each weight
# fragment is loaded once per CU instead of once per M half; natural order
# (the slot plan's skip words are per M half of 2-block waves).
s = open("az_tower16.hip").read()
def rep(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)
rep("  const bool planned = 16 * MBT == T.tile_rows || alt;",
    "  const bool planned = NWM == 2 && (16 * MBT == T.tile_rows || alt);")
rep("""  if (n <= net->alt_max_boards)  // uniform over the launch
    tower16_tile<MBT2, 2, false, DB>(net, boards, x, nullptr, n, H, W, A, bpw2, probs, values, nullptr, 0, err, {});""",
"""  if (n <= net->alt_max_boards) {  // uniform over the launch
    if (threadIdx.x >= 256) return;  // waves 4-7 leave (a barrier counts the waves still running)
    tower16_tile<MBT2, 1, false, DB>(net, boards, x, nullptr, n, H, W, A, bpw2, probs, values, nullptr, 0, err, {});
  }""")
open("az_tower16.hip", "w").write(s)
