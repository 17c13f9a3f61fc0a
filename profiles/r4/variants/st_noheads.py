# diagnostic (wrong outputs): the tower ends after the heads' 1x1 partials --
# the dense heads, softmax and tanh are not run (their share of the tile)
s = open("az_tower16.hip").read()
old = """  if constexpr (ROWS) {
    // per pixel (policy 0, policy 1, value) = 16 partials in order + folded"""
assert old in s
s = s.replace(old, """  if (!ROWS) return;
  if constexpr (ROWS) {
    // per pixel (policy 0, policy 1, value) = 16 partials in order + folded""")
open("az_tower16.hip", "w").write(s)
