# A/B (round 6): the Connect-4 tower without the dual launch (128-row tiles only)
p = 'az_engine.hip'
s = open(p).read()
old = "    if (!rows_tower && tn.tile_rows == 128 && tn.dbuf && tower16_boards_per_tile(HW, 128) == 3 &&"
assert old in s
s = s.replace(old, "    if (false && !rows_tower && tn.tile_rows == 128 && tn.dbuf && tower16_boards_per_tile(HW, 128) == 3 &&")
open(p, 'w').write(s)
