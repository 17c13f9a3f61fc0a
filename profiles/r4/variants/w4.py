# 4 waves (one per SIMD): wave = N quarter over all 8 M blocks of the C4
# tile, so each weight byte is loaded once per tile; natural order (the
# plan's skip masks are per 8-wave M half)
s = open("az_tower16.hip").read()
def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)
rep("const bool planned = 16 * MBT == T.tile_rows;", "const bool planned = NWM == 2 && 16 * MBT == T.tile_rows;")
rep("""    launch_mbw<8, 2, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);
}""", """    launch_mbw<8, 1, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);
}""")
rep("""  auto turn = [&](int k) {
    if ((k ^ mh) & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };""", "  auto turn = [&](int) {};")
open("az_tower16.hip", "w").write(s)
