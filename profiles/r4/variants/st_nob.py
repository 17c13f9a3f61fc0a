# diagnostic (wrong outputs): phase stamps, and no weight stream in the K
# loop (each wave keeps its first k-step's fragments)
exec(open(__file__.replace("st_nob.py", "stamps.py")).read())
s = open("az_tower16.hip").read()
old = "  auto load_bk = [&](int s, uint4(&dst)[4]) {\n"
assert old in s
s = s.replace(old, old + "    if (s >= PF + C0) return;\n")
open("az_tower16.hip", "w").write(s)
