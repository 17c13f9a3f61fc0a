# The assembly K loop prefetching weights 2 k-steps ahead (4 B buffers, +32
# VGPRs; 212 for the 128-row tile) instead of 1.
s = open("az_tower16.hip").read()
assert s.count("#ifndef AZ_KLOOP_PF") == 1
s = "#define AZ_KLOOP_PF 2\n" + s
open("az_tower16.hip", "w").write(s)
