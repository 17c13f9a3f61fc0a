# no priority turn in the K loop
s = open("az_tower16.hip").read()
old = """  auto turn = [&](int k) {
    if ((k ^ mh) & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };"""
assert old in s
s = s.replace(old, "  auto turn = [&](int) {};")
open("az_tower16.hip", "w").write(s)
