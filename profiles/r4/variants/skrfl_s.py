# skrfl for the small tiles only (MBW <= 3: the 9x9 96-row tiles and chess's
# 64-row tiles; the 128-row kernels spill 78-106 VGPRs with scalar dispatch)
s = open("az_tower16.hip").read()
def rep(a, b, cnt=1):
    global s
    assert s.count(a) == cnt, a[:90]
    s = s.replace(a, b)
rep("""  const int skw = planned ? T.skip[mh] : 0;""",
    """  const int skw = MBW <= 3 ? __builtin_amdgcn_readfirstlane(planned ? T.skip[mh] : 0) : (planned ? T.skip[mh] : 0);""")
open("az_tower16.hip", "w").write(s)
