# the phase-priority switch at chunk 1 of tap 5 instead of tap 6's start
s = open("az_tower16.hip").read()
def rep(a, b):
    global s
    assert a in s, a[:80]
    s = s.replace(a, b)
rep("    if (t == 6) prio(!young);\n", "")
rep("""    for (int c = C0; c < 4; ++c) {
      __builtin_amdgcn_sched_barrier(0);
      // main k-step PF ahead""", """    for (int c = C0; c < 4; ++c) {
      __builtin_amdgcn_sched_barrier(0);
      if (c == 1 && t == 5) prio(!young);
      // main k-step PF ahead""")
open("az_tower16.hip", "w").write(s)
