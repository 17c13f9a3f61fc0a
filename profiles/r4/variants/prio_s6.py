# SIMD-pair priority by phase: the younger wave of each SIMD (waves 4-7) at
# priority 1 for taps < 6 of every K loop (and the residual steps), then the
# older at priority 1 -- one scalar s_setprio per switch (the wave index made
# wave-uniform by readfirstlane, so the branch is scalar).  T=0: older first
# all loop long; T=9: younger all loop long
s = open("az_tower16.hip").read()
def rep(a, b):
    global s
    assert a in s, a[:80]
    s = s.replace(a, b)
rep("""  // ---- residual k-steps (static)""", """  const bool young = __builtin_amdgcn_readfirstlane((int)threadIdx.x) >= 256;
  auto prio = [&](bool hi) {
    if (hi) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };
  prio(young == (6 > 0));
  // ---- residual k-steps (static)""")
rep("""    const int m = (skw >> (2 * t)) & 3;
    if (m == 0) tap(t, IC<0>{});""", """    const int m = (skw >> (2 * t)) & 3;
    if (t == 6) prio(!young);
    if (m == 0) tap(t, IC<0>{});""")
rep("""    else tap(t, IC<2>{});
  }
}""", """    else tap(t, IC<2>{});
  }
  __builtin_amdgcn_s_setprio(0);
}""")
open("az_tower16.hip", "w").write(s)
