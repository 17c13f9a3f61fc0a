# A/B (round 6): Connect-4 towers in 96-row tiles of two boards (6 blocks, 3
# per wave; the slot plan's four border blocks) instead of 128-row tiles of
# three: ~30% fewer block-taps per wave (the tile's latency), 1.5x the tiles
# (weight passes) per launch -- with the LRU cache a lane launch is ~120 boards.
p = 'az_tower16.hip'
s = open(p).read()
old = "  if (HW > 64 && HW <= 96) return 192;"
assert old in s
s = s.replace(old, old + "\n  if (HW == 42) return 96;  // variant t96")
open(p, 'w').write(s)
