# diagnostic: per-slot select phase stamps (profiles/sel_stamps.py reads them)
s = open("az_tree.hip").read()
s = "#define AZ_SEL_STAMPS 1\n" + s
open("az_tree.hip", "w").write(s)
