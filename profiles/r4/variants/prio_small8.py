# the phase-priority switch at tap 8 for the small tiles (MBW <= 3: 9x9's
# 96-row tiles, chess's 64-row tiles), tap 6 for Connect-4's 128-row tiles
s = open("az_tower16.hip").read()
old = "    if (t == 6) prio(!young);"
assert old in s
s = s.replace(old, "    if (t == (MBW <= 3 ? 8 : 6)) prio(!young);")
open("az_tower16.hip", "w").write(s)
