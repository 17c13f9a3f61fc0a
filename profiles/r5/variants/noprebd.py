# The stem's board loads after the plan load (round 4's dependent order)
# instead of beside it.
s = open("az_tower16.hip").read()
old = "      for (int k = 0; k < kPre; ++k) pre[k] = gld(boards + b0 + min(k, nbrd - 1));"
assert s.count(old) == 1
s = s.replace(old, "      for (int k = 0; k < kPre; ++k) pre[k] = Board{};")
old = "          if (nbrd <= kPre) bd[i] = bi == 0 ? pre[0] : bi == 1 ? pre[1] : pre[2];"
assert s.count(old) == 1
s = s.replace(old, "          if (false) bd[i] = pre[0];")
open("az_tower16.hip", "w").write(s)
