# pairl1 with the priority alternation keyed on the SIMD partner (wave >> 2)
exec(open("/root/repo/profiles/r4/variants/pairl1.py").read())
s = open("az_tower16.hip").read()
import re
n = s.count("lane, mh, skw")
s = s.replace("lane, mh, skw", "lane, (int)(threadIdx.x >> 8), skw")
assert n >= 4, n
open("az_tower16.hip", "w").write(s)
