# the value dense's weights (wv1, 43 KB for 6x7) not in the kernel-start blob
# DMA: they stream into X's dead tile during the last conv2 (wv1_xtile)
s = open("az_engine.hip").read()
old = "      for (int i = 0; i < (rows_tower ? 1 : 3) && !found; ++i)"
assert old in s
s = s.replace(old, "      for (int i = rows_tower ? 0 : 1; i < (rows_tower ? 1 : 3) && !found; ++i)")
open("az_engine.hip", "w").write(s)
