# M halves by wave parity (mh = wave & 1, nq = wave >> 1): the two waves that
# load the same weight fragments (one N quarter, both M halves) sit on
# different SIMDs as both older (waves 0-3) or both younger (4-7), so they
# run in step and the second request finds the line in the CU's L1
s = open("az_tower16.hip").read()
old = "const int mh = wave >> 2, nq = wave & 3"
assert old in s
s = s.replace(old, "const int mh = wave & 1, nq = wave >> 1")
open("az_tower16.hip", "w").write(s)
