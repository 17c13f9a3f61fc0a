# weights two k-steps ahead (ring of 4) in the K loops of tiles with at most
# 3 blocks per wave (9x9's 96-row tiles, chess's 64-row tiles: no spill there)
s = open("az_tower16.hip").read()
def rep(a, b):
    global s
    assert a in s, a[:80]
    s = s.replace(a, b)
rep("  constexpr int PF = 1, NB = 2;", "  constexpr int PF = (MBW <= 3 && C0 == 0) ? 2 : 1, NB = 2 * PF;")
rep('''  static_assert(PF == 1, "one prefetched k-step");
  if (pre) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[C0 % NB][q] = pre[q];
  } else {
    load_bk(C0, bq[C0 % NB]);
  }''', '''  if (pre) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[C0 % NB][q] = pre[q];
  } else {
    load_bk(C0, bq[C0 % NB]);
  }
  if (PF == 2) load_bk(C0 + 1, bq[(C0 + 1) % NB]);''')
open("az_tower16.hip", "w").write(s)
