# A/B (round 6): MT twist batches of 16 words (39 round trips) instead of 48
p = 'az_tree.hip'
s = open(p).read()
old = "  constexpr int kTwistB = 48;"
assert s.count(old) == 1
s = s.replace(old, "  constexpr int kTwistB = 16;")
open(p, 'w').write(s)
