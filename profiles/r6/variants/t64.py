# A/B (round 6): Connect-N board towers in 64-row tiles of one board
# (MBT 4, 8 waves of 2 blocks: half the K-loop latency per tile, 1.5x the
# MFMAs per board) instead of 128-row tiles of three -- with the LRU cache a
# lane launch holds ~120 boards, so the tile's latency, not the CUs, bounds it.
p = 'az_tower16.hip'
s = open(p).read()
old = '''  else
    launch_mbw<8, 2, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);
}'''
new = '''  else if (tile_rows == 128 && H * W <= 64)
    launch_mbw<4, 2, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);
  else
    launch_mbw<8, 2, false>(net, staged, dbuf, boards, x, nullptr, count, n_max, H, W, A, probs, values, nullptr, 0,
                            err, s);
}'''
assert old in s
s = s.replace(old, new)
open(p, 'w').write(s)
