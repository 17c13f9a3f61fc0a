# The duplicate-board resolution as its own one-block launch after select
# (round 4's shape) instead of the select launch's last block.
s = open("az_tree.hip").read()
old_k = """template <bool NOISE>
__global__ __launch_bounds__(kGameBlock) void select_kernel(GameCfg g, TreeDev t, CacheDev c) {
  select_body<NOISE>(g, t, c);
  dedup_tail(t, c);
}
template <int L, bool NOISE>
__global__ __launch_bounds__(kGameBlock) void select_group_kernel(GameCfg g, TreeDev t, CacheDev c) {
  select_group_body<L, NOISE>(g, t, c);
  dedup_tail(t, c);
}"""
assert s.count(old_k) == 1
s = s.replace(old_k, """template <bool NOISE>
__global__ __launch_bounds__(kGameBlock) void select_kernel(GameCfg g, TreeDev t, CacheDev c) {
  select_body<NOISE>(g, t, c);
}
template <int L, bool NOISE>
__global__ __launch_bounds__(kGameBlock) void select_group_kernel(GameCfg g, TreeDev t, CacheDev c) {
  select_group_body<L, NOISE>(g, t, c);
}
__global__ __launch_bounds__(kGameBlock) void dedup_kernel(TreeDev t, CacheDev c) { dedup_tail(t, c); }""")
old_l = """    default: select_kernel<false><<<game_blocks(g.slots), kGameBlock, 0, s>>>(g, t, c); break;
  }
}"""
assert s.count(old_l) == 1
s = s.replace(old_l, """    default: select_kernel<false><<<game_blocks(g.slots), kGameBlock, 0, s>>>(g, t, c); break;
  }
  dedup_kernel<<<1, kGameBlock, 0, s>>>(t, c);
}""")
open("az_tree.hip", "w").write(s)
