# Connect-4 on 192-row in-place tiles (four boards per workgroup, the 9x9
# form) instead of 128-row double-buffered tiles of three: half the weight
# stream per board, fewer and longer tiles per launch.
s = open("az_tower16.hip").read()
old = "  if (HW > 64 && HW <= 96) return 192;"
assert s.count(old) == 1
s = s.replace(old, "  if ((HW > 64 && HW <= 96) || HW == 42) return 192;")
open("az_tower16.hip", "w").write(s)
