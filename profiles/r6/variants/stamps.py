# diagnostic: phase clocks (profiles/tower_stamps.py reads them)
s = open("az_tower16.hip").read()
s = "#define AZ_T16_STAMPS 1\n" + s
open("az_tower16.hip", "w").write(s)
