# Diagnostic build: select-phase and dedup-tail stamps (profiles/sel_stamps.py).
s = open("az_tree.hip").read()
s = "#define AZ_SEL_STAMPS 1\n" + s
open("az_tree.hip", "w").write(s)
