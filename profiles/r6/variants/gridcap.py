# A/B (round 6): Connect-4's dual tower launch with a grid of at most 256
# workgroups, each looping over tiles (tile += gridDim.x), instead of one
# workgroup per possible tile of the lane (683 at 1365 slots, ~620 of them
# leaving at once at the ~122 live boards of a cached simulation)
p = 'az_tower16.hip'
s = open(p).read()
def rep(old, new, cnt=1):
    global s
    assert s.count(old) == cnt, (old, s.count(old))
    s = s.replace(old, new)
rep("""                                             int first_chunk, unsigned long long* __restrict__ err,
                                             TowerLeaves lv) {
  constexpr int MBW = MBT / NWM;  // M blocks per wave""",
"""                                             int first_chunk, unsigned long long* __restrict__ err,
                                             TowerLeaves lv, int tile = -1) {
  constexpr int MBW = MBT / NWM;  // M blocks per wave""")
rep("""  const int b0 = blockIdx.x * bpw;
  if (b0 >= n) return;  // block-uniform""", """  const int b0 = (tile >= 0 ? tile : (int)blockIdx.x) * bpw;
  if (b0 >= n) return;  // block-uniform""")
rep("""  const int n = count ? *count : n_static;
  if (n <= net->alt_max_boards)  // uniform over the launch
    tower16_tile<MBT2, 2, false, DB>(net, boards, x, nullptr, n, H, W, A, bpw2, probs, values, nullptr, 0, err, {});
  else
    tower16_tile<MBT, 2, false, DB>(net, boards, x, nullptr, n, H, W, A, bpw, probs, values, nullptr, 0, err, {});""",
"""  const int n = count ? *count : n_static;
  const bool small = n <= net->alt_max_boards;  // uniform over the launch
  const int per = small ? bpw2 : bpw;
  for (int tile = blockIdx.x; tile * per < n; tile += gridDim.x) {  // block-uniform
    if (small)
      tower16_tile<MBT2, 2, false, DB>(net, boards, x, nullptr, n, H, W, A, bpw2, probs, values, nullptr, 0, err, {}, tile);
    else
      tower16_tile<MBT, 2, false, DB>(net, boards, x, nullptr, n, H, W, A, bpw, probs, values, nullptr, 0, err, {}, tile);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();  // the tile's LDS reads done before the next tile's writes
  }""")
rep("""    const int grid = (n_max + bpw2 - 1) / bpw2;
    const size_t bytes = std::max(""", """    const int grid = std::min((n_max + bpw2 - 1) / bpw2, 256);
    const size_t bytes = std::max(""")
open(p, 'w').write(s)
