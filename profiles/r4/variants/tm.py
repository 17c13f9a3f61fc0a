# term-major k-steps (t1*B0 over every block, then t0*b1, then t0*B0) on a
# single-buffered ring: measured 1% slower in the product (13 spills)
s = open("az_tower16.hip").read()
a = s.index("  // activation fragments in a ring of RING M blocks:")
b = s.index("#pragma unroll\n  for (int k = 0; k < PF; ++k) load_bk(C0 + k, bq[(C0 + k) % NB]);")
new = '''  uint4 aq[MBW][2];
  auto load_t = [&](int chunk, int mb, int term) {
    aq[mb][term] = *reinterpret_cast<const uint4*>(actb + aaddr[mb] + 64 * chunk + 256 * term);
  };
  auto kstep = [&](t_f4(&C)[MBW][2], const uint4(&b)[4], int next_chunk, auto skc, auto skn) {
    constexpr int SKC = decltype(skc)::value, SKN = decltype(skn)::value;
    const t_h8 B0[2] = {__builtin_bit_cast(t_h8, b[0]), __builtin_bit_cast(t_h8, b[2])};
    const t_h8 B1[2] = {__builtin_bit_cast(t_h8, b[1]), __builtin_bit_cast(t_h8, b[3])};
#pragma unroll
    for (int term = 0; term < 3; ++term) {
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        if (((SKC >> mb) & 1) == 0) {
          const t_h8 a = __builtin_bit_cast(t_h8, aq[mb][term == 0 ? 1 : 0]);
#pragma unroll
          for (int nb = 0; nb < 2; ++nb)
            C[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(term == 1 ? B1[nb] : B0[nb], a, C[mb][nb], 0, 0, 0);
        }
        if (term != 1 && next_chunk >= 0 && ((SKN >> mb) & 1) == 0) load_t(next_chunk, mb, term == 0 ? 1 : 0);
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x0020, 4, 0);
#pragma unroll
    for (int term = 0; term < 3; ++term)
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) {
        if (((SKC >> mb) & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x0008, 2, 0);
        if (term != 1 && next_chunk >= 0 && ((SKN >> mb) & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
      }
  };

'''
s = s[:a] + new + s[b:]
def rep(old, new_):
    global s
    assert old in s, old
    s = s.replace(old, new_)
rep('''#pragma unroll
  for (int mb = 0; mb < RING; ++mb) load_a1(C0, mb);''', '''#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    load_t(C0, mb, 0);
    load_t(C0, mb, 1);
  }''')
rep('''    if (s + 1 == R) set_tap(0, 0, LAG ? MBW - 1 : RING);
    kstep(accr, bq[s % NB], s, s + 1 == R ? 0 : s + 1, IC<0>{}, IC<0>{}, s == 0);''', '''    if (s + 1 == R) set_tap(0, 0, MBW);
    kstep(accr, bq[s % NB], s + 1 == R ? C0 : s + 1, IC<0>{}, IC<0>{});''')
a = s.index("      // the tap's high blocks (first k-step; tap 0 after the residual steps)")
b = s.index("    }\n  };\n#pragma unroll 1\n  for (int t = 0; t < 9; ++t) {")
s = s[:a] + '''      if (c < 3) {
        kstep(acc, bq[c % NB], c + 1, skc, skc);
      } else if (t < 8) {
        set_tap(t + 1, 0, MBW);
        kstep(acc, bq[c % NB], C0, skc, IC<0>{});
      } else {
        kstep(acc, bq[c % NB], -1, skc, IC<0>{});
      }
''' + s[b:]
open("az_tower16.hip", "w").write(s)
