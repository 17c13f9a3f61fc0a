# diagnostic (wrong outputs): the tower ends after the pf/vf features (no
# dense heads, no softmax)
s = open("az_tower16.hip").read()
old = "  T16_STAMP(44);"
assert old in s
s = s.replace(old, old + "\n  if (!ROWS) return;")
open("az_tower16.hip", "w").write(s)
