# chess lanes' policy dense at 4 boards per workgroup (NB = 1: 960 workgroups at 128 boards) instead of 8
import re
p = "az_nn.hip"
s = open(p).read()
a = "policy_dense_kernel<128, 2><<<dim3((A + 63) / 64, (n_max + 7) / 8), 256, 0, s>>>"
assert s.count(a) == 1
s = s.replace(a, "policy_dense_kernel<128, 1><<<dim3((A + 63) / 64, (n_max + 3) / 4), 256, 0, s>>>")
open(p, "w").write(s)
