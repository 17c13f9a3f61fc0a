# Chess's 64-row tiles with the runtime skip word (three tap bodies per K
# loop, as before round 5's compile-time 0).
s = open("az_tower16.hip").read()
old = "  const int skw = (ROWS && 16 * MBT != 128) ? 0 : planned ? T.skip[mh] : 0;"
assert s.count(old) == 1
s = s.replace(old, "  const int skw = planned ? T.skip[mh] : 0;")
open("az_tower16.hip", "w").write(s)
