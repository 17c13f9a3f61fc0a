# Diagnostic (wrong outputs): the assembly K loop without its weight loads
# (every buffer_load of a B fragment commented out), to see how much of the
# tile the weight stream costs -- chess's 2-block waves load twice the
# weight bytes per MFMA of Connect-4's 4-block waves.
s = open("az_kloop_asm.h").read()
n = s.count("buffer_load_dwordx4 %[b")
assert n > 100
s = s.replace("buffer_load_dwordx4 %[b", "; nob %[b")
open("az_kloop_asm.h", "w").write(s)
m = open("Makefile").read()
m = m.replace("az_kloop_asm.h: gen_kloop_asm.py\n\tpython3 gen_kloop_asm.py\n", "az_kloop_asm.h:\n\ttrue\n")
open("Makefile", "w").write(m)
