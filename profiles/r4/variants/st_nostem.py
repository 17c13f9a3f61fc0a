# diagnostic (wrong outputs): the Connect-N stem builds no operand and issues
# no MFMA (its share of the tile; the boards are still read)
s = open("az_tower16.hip").read()
old = """          uint4 a0, a1;
          split_u8(v, a0, a1);"""
assert old in s
s = s.replace(old, """          uint4 a0, a1;
          split_u8(v, a0, a1);
          if (v[0] != 12345.f) continue;""")
open("az_tower16.hip", "w").write(s)
