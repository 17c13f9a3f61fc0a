# The assembly K loop prefetching weights 1 k-step ahead (2 B buffers).
s = open("az_tower16.hip").read()
assert s.count("#ifndef AZ_KLOOP_PF") == 1
s = "#define AZ_KLOOP_PF 1\n" + s
open("az_tower16.hip", "w").write(s)
