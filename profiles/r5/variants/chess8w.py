# Chess's one-board 64-row tiles in 8 waves (2 blocks per wave, 2 waves per
# SIMD: round 4's shape) instead of 16.
s = open("az_tower16.hip").read()
old = "    launch_mbw<4, 4, true>(net, staged, dbuf, nullptr, nullptr, static_cast<const uint4*>(rows), count, n_max, H, W,"
assert s.count(old) == 1
s = s.replace(old, "    launch_mbw<4, 2, true>(net, staged, dbuf, nullptr, nullptr, static_cast<const uint4*>(rows), count, n_max, H, W,")
open("az_tower16.hip", "w").write(s)
