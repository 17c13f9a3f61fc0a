# A/B (round 6): no per-simulation dedup of identical leaves -- a miss takes
# its own evaluator row at once (a board two slots reach in one simulation is
# evaluated twice: the same outputs, so the same search), and the select
# launch loses the dedup table's round trips, the per-block done count and
# the last block's tail
p = 'az_tree.hip'
s = open(p).read()
start = s.index("  wave_count(t.miss_count);\n  const uint64_t tag = ((uint64_t)t.epoch << 32)")
end = s.index("// ---------------------------------------------------- Dirichlet root noise")
s = s[:start] + """  wave_count(t.miss_count);
  const int row = wave_claim(t.nn_count);
  t.nn_board[row] = b;
  t.eval_src[q] = -(row + 1);
  wave_stat(t, kStatNNEvals);
}

""" + s[end:]
old = """__device__ __forceinline__ void dedup_tail(const TreeDev& t, const CacheDev& c) {
  if (!c.enabled) return;  // uniform"""
assert s.count(old) == 1
s = s.replace(old, """__device__ __forceinline__ void dedup_tail(const TreeDev& t, const CacheDev& c) {
  return;""")
old = """    tag0 = __hip_atomic_load(t.step_tag + ((uint32_t)h & t.step_mask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
"""
assert s.count(old) == 1
s = s.replace(old, "")
open(p, 'w').write(s)
