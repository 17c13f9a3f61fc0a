# Chess's one-board 64-row tiles in 4 waves (one per SIMD, 4 blocks x 32
# channels each: each weight fragment loaded once per tile instead of by a
# wave pair) instead of 8 waves of 2 blocks.
s = open("az_tower16.hip").read()
old = "    launch_mbw<4, 2, true>(net, staged, dbuf, nullptr, nullptr, static_cast<const uint4*>(rows), count, n_max, H, W,"
assert s.count(old) == 1
s = s.replace(old, "    launch_mbw<4, 1, true>(net, staged, dbuf, nullptr, nullptr, static_cast<const uint4*>(rows), count, n_max, H, W,")
open("az_tower16.hip", "w").write(s)
