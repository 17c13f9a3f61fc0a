# the wave's tap-skip word through readfirstlane: T.skip[mh] is indexed by
# the wave parity, which the compiler cannot prove uniform, so the three tap
# bodies were dispatched as an exec-masked if-chain (saveexec / execz skips,
# and register copies plus an LDS wait at every tap's back-edge); as an SGPR
# the dispatch becomes scalar branches
s = open("az_tower16.hip").read()
def rep(a, b, cnt=1):
    global s
    assert s.count(a) == cnt, a[:90]
    s = s.replace(a, b)
rep("""  const int skw = planned ? T.skip[mh] : 0;""",
    """  const int skw = __builtin_amdgcn_readfirstlane(planned ? T.skip[mh] : 0);""")
open("az_tower16.hip", "w").write(s)
