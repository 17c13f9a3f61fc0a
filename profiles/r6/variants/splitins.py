# Diagnostic (round 6): the Connect-4 cache inserts as a launch of their own
# right after the expand on the lane's stream, so a kernel trace times the
# expand half and the insert half separately (same work, one more launch)
p = 'az_tree.hip'
s = open(p).read()
old = '''    if (ins) expand_kernel<16, true, 1><<<grid, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);
    else expand_kernel<16, false, 1><<<grid, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);'''
assert old in s
s = s.replace(old, '''    expand_kernel<16, false, 1><<<eb, kGameBlock, 0, s>>>(g, t, c, probs, values, eb);
    if (ins) expand_kernel<16, true, 1><<<grid - eb, kGameBlock, 0, s>>>(g, t, c, probs, values, 0);''')
open(p, 'w').write(s)
