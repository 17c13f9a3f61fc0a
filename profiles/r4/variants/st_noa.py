# diagnostic (wrong outputs): phase stamps, and the activation fragments read
# only for the first chunk of each tap
exec(open(__file__.replace("st_noa.py", "stamps.py")).read())
s = open("az_tower16.hip").read()
old = "  auto load_a1 = [&](int chunk, int mb) {\n"
assert old in s
s = s.replace(old, old + "    if (chunk > C0) return;\n")
open("az_tower16.hip", "w").write(s)
