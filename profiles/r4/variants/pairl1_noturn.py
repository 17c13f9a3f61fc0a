# pairl1 without the per-k-step priority alternation
exec(open("/root/repo/profiles/r4/variants/pairl1.py").read())
s = open("az_tower16.hip").read()
old = """  auto turn = [&](int k) {
    if ((k ^ mh) & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };"""
assert old in s
s = s.replace(old, "  auto turn = [&](int) {};")
open("az_tower16.hip", "w").write(s)
