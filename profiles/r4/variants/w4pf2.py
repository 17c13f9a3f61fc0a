# w4 with the weight fragments two k-steps ahead (ring of 4)
exec(open(__file__.replace("w4pf2.py", "w4.py")).read())
s = open("az_tower16.hip").read()
old = "  constexpr int PF = 1, NB = 2;"
assert old in s
s = s.replace(old, "  constexpr int PF = 2, NB = 4;")
open("az_tower16.hip", "w").write(s)
