# no per-k-step turn; the second-dispatched half (waves 4-7) at priority 1 for
# the whole kernel (MI355X_MICROARCH.md, two waves per SIMD, item 4)
s = open("az_tower16.hip").read()
old = """  auto turn = [&](int k) {
    if ((k ^ mh) & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };"""
assert old in s
s = s.replace(old, "  auto turn = [&](int) {};")
s = s.replace("  __builtin_amdgcn_s_setprio(0);\n}", "}")
old = "  const int mh = wave >> 2, nq = wave & 3, r16 = lane & 15, gq = lane >> 4;"
assert old in s
s = s.replace(old, old + "\n  if (__builtin_amdgcn_readfirstlane(wave) >= 4) __builtin_amdgcn_s_setprio(1);")
open("az_tower16.hip", "w").write(s)
