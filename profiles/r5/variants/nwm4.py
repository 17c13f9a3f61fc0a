# The Connect-4 128-row tower tile in 16 waves (4 M quarters x 4 N quarters,
# four waves per SIMD at <= 128 VGPRs) instead of 8: more waves to hide the
# K loop's latencies; each weight fragment then feeds 2 M blocks per wave
# (L1 -> VGPR weight traffic x2; L2 -> L1 unchanged when the 4 waves of an
# N quarter run in step).  The slot plan's border blocks are blocks 0-1 of
# each M half = M quarters 0 and 2.
s = open("az_tower16.hip").read()
def rep(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)
rep("  const int skw = planned ? T.skip[mh] : 0;",
    "  const int skw = planned ? (NWM == 2 ? T.skip[mh] : (mh & 1) ? 0 : T.skip[mh >> 1]) : 0;")
rep("""  else
    launch_mbw<8, 2, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);""", """  else
    launch_mbw<8, 4, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);""")
open("az_tower16.hip", "w").write(s)
