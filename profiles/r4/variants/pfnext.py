# each K loop's last k-step prefetches the NEXT K loop's first weight
# fragments (the ring owned by the kernel), so their L2 latency runs under
# the epilogue and barrier: measured 4% SLOWER isolated, -2% in-bench
s = open("az_tower16.hip").read()
def rep(a, b, cnt=1):
    global s
    assert s.count(a) == cnt, a[:100]
    s = s.replace(a, b)
rep("""                                       int zrow, int nq, int lane, int mh, int skw, int res_shift = 0,
                                       Mid mid = Mid{}) {""", """                                       int zrow, int nq, int lane, int mh, int skw, uint4 (&bq)[2][4],
                                       bool prefetched, const uint4* wnext, int next_ks, int res_shift = 0,
                                       Mid mid = Mid{}) {""")
rep("""  uint4 bq[NB][4];
  // k-step s of the phase""", """  // k-step s of the phase""")
rep("""  const int voff = ((nq * 2) * 2 * 64 + lane) * 16;
  auto load_bk = [&](int s, uint4(&dst)[4]) {""", """  const auto rs_n = __builtin_amdgcn_make_buffer_rsrc((void*)(wnext ? wnext : wmain), (short)0, 0x7fffffff,
                                                      0x00020000);
  const int voff = ((nq * 2) * 2 * 64 + lane) * 16;
  auto load_next = [&](uint4(&dst)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      dst[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_n, voff + q * 1024, next_ks * 16384, 0));
  };
  auto load_bk = [&](int s, uint4(&dst)[4]) {""")
rep("""#pragma unroll
  for (int k = 0; k < PF; ++k) load_bk(C0 + k, bq[(C0 + k) % NB]);""", """  if (!prefetched) load_bk(C0, bq[0]);""")
rep("""      if (c + PF < 4 || t < 8) load_bk(R + ahead, bq[(c + PF) % NB]);""", """      if (c + PF < 4 || t < 8) load_bk(R + ahead, bq[(c + PF) % NB]);
      else if (wnext) load_next(bq[(c + PF) % NB]);""")
rep("""    if (first_chunk == 2) k_loop<MBW, 0, 2>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, mh, skw);
    else k_loop<MBW, 0>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, mh, skw);""", """    if (first_chunk == 2) k_loop<MBW, 0, 2>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, mh, skw, bq, false, first_w, first_ks);
    else k_loop<MBW, 0>(bufH, T.stem_k, nullptr, acc, acc, yx, H, W, zH, nq, lane, mh, skw, bq, false, first_w, first_ks);""")
rep("""    if constexpr (DB) k_loop<MBW, 0>(bufX, T.k1[d], nullptr, acc, acc, yx, H, W, zX, nq, lane, mh, skw);
    else k_loop<MBW, 4>(bufX, T.k1[d], T.k2[d], acc, accr_, yx, H, W, zX, nq, lane, mh, skw);""", """    if constexpr (DB) k_loop<MBW, 0>(bufX, T.k1[d], nullptr, acc, acc, yx, H, W, zX, nq, lane, mh, skw, bq, true, T.k2[d], 36);
    else k_loop<MBW, 4>(bufX, T.k1[d], T.k2[d], acc, accr_, yx, H, W, zX, nq, lane, mh, skw, bq, true, T.k2[d], 0);""")
rep("""      k_loop<MBW, 4>(bufH, T.k2[d], T.k2[d], acc, acc, yx, H, W, zH, nq, lane, mh, skw, -(TR + kZeroRows), mid);""", """      k_loop<MBW, 4>(bufH, T.k2[d], T.k2[d], acc, acc, yx, H, W, zH, nq, lane, mh, skw, bq, true, d + 1 < depth ? T.k1[d + 1] : nullptr, 0, -(TR + kZeroRows), mid);""")
rep("""      k_loop<MBW, 0>(bufH, T.k2[d], nullptr, accr, accr, yx, H, W, zH, nq, lane, mh, skw);""", """      k_loop<MBW, 0>(bufH, T.k2[d], nullptr, accr, accr, yx, H, W, zH, nq, lane, mh, skw, bq, true, d + 1 < depth ? T.k2[d + 1] : nullptr, 36);""")
rep("""  float4 yv[2 * MBW];
""", """  float4 yv[2 * MBW];
  uint4 bq[2][4];
  const uint4* const first_w = T.depth > 0 ? (DB ? T.k1[0] : T.k2[0]) : nullptr;
  const int first_ks = DB ? 0 : 36;
""")
old = """      for (int q = 0; q < 4; ++q) bs2[ks][q] = gld(ws + (size_t)ks * 1024 + q * 64);"""
rep(old, old + """
    if (first_w) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)first_w, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bq[0][q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((nq * 2) * 2 * 64 + lane) * 16 + q * 1024, first_ks * 16384, 0));
    }""")
open("az_tower16.hip", "w").write(s)
