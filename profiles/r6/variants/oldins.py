# A/B (round 6): Connect-N cache inserts published behind a full __threadfence
# per thread (round 5) instead of one release per insert block
p = 'az_tree.hip'
s = open(p).read()
old = '''  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (idx < 0) return;
  atomicExch(c.state + idx, word);'''
assert old in s
s = s.replace(old, '''  if (idx < 0) return;
  __threadfence();
  atomicExch(c.state + idx, word);''')
open(p, 'w').write(s)
