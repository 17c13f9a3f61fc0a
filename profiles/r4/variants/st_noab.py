# diagnostic (wrong outputs): stamps, no weight stream and no activation reads past each tap's first chunk
s = open("az_tower16.hip").read()
s = "#define AZ_T16_STAMPS 1\n" + s
old = "  auto load_bk = [&](int s, uint4(&dst)[4]) {\n"
assert old in s
s = s.replace(old, old + "    if (s >= PF + C0) return;\n")
old = "  auto load_a1 = [&](int chunk, int mb) {\n"
assert old in s
s = s.replace(old, old + "    if (chunk > C0) return;\n")
open("az_tower16.hip", "w").write(s)
