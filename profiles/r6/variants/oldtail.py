# A/B (round 6): the select launch's block-done protocol as in round 5 (a full
# __threadfence per wave before the count, another in the last block)
for p, tag in (('az_tree.hip', 'threadIdx.x == 0'), ('az_chess_mcts.hip', 'lane == 0')):
    s = open(p).read()
    i = s.index('  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n  __syncthreads();\n  if (%s) {' % tag)
    j = s.index('  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");\n  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");', i)
    j2 = j + len('  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");\n  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");')
    old = ('  __threadfence();\n  __syncthreads();\n  if (%s) last = atomicAdd(t.sel_done, 1u) == gridDim.x - 1;\n'
           '  __syncthreads();\n  if (!last) return;  // block-uniform\n  __threadfence();') % tag
    s = s[:i] + old + s[j2:]
    open(p, 'w').write(s)
