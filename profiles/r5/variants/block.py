# The assembly K loop in block-major order (gen_kloop_asm.group_asm).
s = open("az_tower16.hip").read()
assert s.count("#ifndef AZ_KLOOP_TERM") == 1
s = "#define AZ_KLOOP_TERM 0\n" + s
open("az_tower16.hip", "w").write(s)
