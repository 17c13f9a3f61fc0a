# the SIMD pair's priority turn as designed: the turn's predicate made
# wave-uniform (readfirstlane), so the compiler branches on a scalar and only
# the chosen s_setprio executes (with mh in a VGPR both setprio instructions
# of the exec-masked branch run: every wave ends each k-step at the same priority)
s = open("az_tower16.hip").read()
old = """  auto turn = [&](int k) {
    if ((k ^ mh) & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };"""
assert old in s
s = s.replace(old, """  auto turn = [&](int k) {
    if (__builtin_amdgcn_readfirstlane((k ^ mh) & 1)) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };""")
open("az_tower16.hip", "w").write(s)
