# the tap-skip word wave-uniform (readfirstlane): the per-tap body dispatch
# becomes a scalar branch instead of an exec-masked one
s = open("az_tower16.hip").read()
old = "  const int skw = T.skip[mh];"
assert old in s
s = s.replace(old, "  const int skw = __builtin_amdgcn_readfirstlane(T.skip[mh]);")
open("az_tower16.hip", "w").write(s)
