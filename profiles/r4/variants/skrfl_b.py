# skrfl with the tap dispatch as m == 1 / m == 2 / else
s = open("az_tower16.hip").read()
def rep(a, b, cnt=1):
    global s
    assert s.count(a) == cnt, a[:90]
    s = s.replace(a, b)
rep("""  const int skw = planned ? T.skip[mh] : 0;""",
    """  const int skw = __builtin_amdgcn_readfirstlane(planned ? T.skip[mh] : 0);""")
rep("""    if (m == 0) tap(t, IC<0>{});
    else if (m == 1) tap(t, IC<1>{});
    else tap(t, IC<2>{});""", """    if (m == 1) tap(t, IC<1>{});
    else if (m == 2) tap(t, IC<2>{});
    else tap(t, IC<0>{});""")
open("az_tower16.hip", "w").write(s)
