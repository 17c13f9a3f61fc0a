# The assembly K loop in term-major order (gen_kloop_asm.term_group_asm):
# an accumulator's three dependent MFMAs 2*MBW instructions apart.
s = open("az_tower16.hip").read()
assert s.count("#ifndef AZ_KLOOP_TERM") == 1
s = "#define AZ_KLOOP_TERM 1\n" + s
open("az_tower16.hip", "w").write(s)
