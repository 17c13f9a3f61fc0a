# the next K loop's first weight k-step loaded right after a K loop, before the
# epilogue's stores and barrier (into registers the next loop's prologue
# takes): equal isolated, -0.5% in-bench (profiles/r4/shape_runs/ab_pfpost.txt)
s = open("az_tower16.hip").read()
def rep(a, b, cnt=1):
    global s
    assert s.count(a) == cnt, a[:90]
    s = s.replace(a, b)
rep("""                                       int zrow, int nq, int lane, int skw, int res_shift = 0,
                                       Mid mid = Mid{}) {""", """                                       int zrow, int nq, int lane, int skw, const uint4* pre,
                                       int res_shift = 0, Mid mid = Mid{}) {""")
rep("""#pragma unroll
  for (int k = 0; k < PF; ++k) load_bk(C0 + k, bq[(C0 + k) % NB]);
  if (R) set_own(0, MBW);""", """  if (pre) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[C0 % NB][q] = pre[q];
  } else {
    load_bk(C0, bq[C0 % NB]);
  }
  if (R) set_own(0, MBW);""")
rep("""  float4 yv[2 * MBW];
""", """  float4 yv[2 * MBW];
  uint4 pre[4];
  auto prefetch = [&](const uint4* pack, int ks) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)pack, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      pre[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rs, ((nq * 2) * 2 * 64 + lane) * 16 + q * 1024, ks * 16384, 0));
  };
""")
rep("""    if (first_chunk == 2) k_loop<MBW, 0, 2>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, skw);
    else k_loop<MBW, 0>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, skw);""", """    if (first_chunk == 2) k_loop<MBW, 0, 2>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, skw, nullptr);
    else k_loop<MBW, 0>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, skw, nullptr);
    prefetch(DB ? T.k1[0] : T.k2[0], DB ? 0 : 36);""")
old = """      for (int q = 0; q < 4; ++q) bs2[ks][q] = gld(ws + (size_t)ks * 1024 + q * 64);"""
rep(old, old + """
    prefetch(DB ? T.k1[0] : T.k2[0], DB ? 0 : 36);""")
rep("""    if constexpr (DB) k_loop<MBW, 0>(bufX, T.k1[d], nullptr, acc, acc, yx, H, W, zX, nq, lane, skw);
    else k_loop<MBW, 4>(bufX, T.k1[d], T.k2[d], acc, accr_, yx, H, W, zX, nq, lane, skw);""", """    if constexpr (DB) k_loop<MBW, 0>(bufX, T.k1[d], nullptr, acc, acc, yx, H, W, zX, nq, lane, skw, pre);
    else k_loop<MBW, 4>(bufX, T.k1[d], T.k2[d], acc, accr_, yx, H, W, zX, nq, lane, skw, pre);""")
rep("""    anyH = store_layer<MBW>(bufH, HW, W, yx, cq0, yv, sm, par, sm.sc[1], nbrd, err);""", """    prefetch(T.k2[d], DB ? 36 : 0);
    anyH = store_layer<MBW>(bufH, HW, W, yx, cq0, yv, sm, par, sm.sc[1], nbrd, err);""")
rep("""      k_loop<MBW, 4>(bufH, T.k2[d], T.k2[d], acc, acc, yx, H, W, zH, nq, lane, skw, -(TR + kZeroRows), mid);""", """      k_loop<MBW, 4>(bufH, T.k2[d], T.k2[d], acc, acc, yx, H, W, zH, nq, lane, skw, pre, -(TR + kZeroRows), mid);""")
rep("""      k_loop<MBW, 0>(bufH, T.k2[d], nullptr, accr, accr, yx, H, W, zH, nq, lane, skw);""", """      k_loop<MBW, 0>(bufH, T.k2[d], nullptr, accr, accr, yx, H, W, zH, nq, lane, skw, pre);""")
rep("""      anyX = store_layer<MBW>(bufX, HW, W, yx, cq0, yv, sm, par, sm.sc[0], nbrd, err);""", """      prefetch(DB ? T.k1[d + 1] : T.k2[d + 1], DB ? 0 : 36);
      anyX = store_layer<MBW>(bufX, HW, W, yx, cq0, yv, sm, par, sm.sc[0], nbrd, err);""")
open("az_tower16.hip", "w").write(s)
