# Two workgroups per CU for Connect-4 (VERDICT r4's "LDS-halved tile"):
# 96-row in-place tiles of two boards with the small staging (LDS <= 80 KB
# per workgroup), the kernel compiled for 4 waves per SIMD (<= 128 VGPRs),
# 1-step weight prefetch -- so one tile's stem, epilogues and heads overlap
# the other's K loop.  The price: 84 of 96 rows live (vs 126 of 128).
import re
s = open("az_tower16.hip").read()
def rep(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)
rep("  if (HW > 128) return 0;\n", "  if (HW > 128) return 0;\n  if (HW == 42) return 96;\n")
rep("__global__ __launch_bounds__(NWM * 256, NWM) void tower16_kernel(",
    "__global__ __launch_bounds__(NWM * 256, (MBT == 6 && !DB) ? 4 : NWM) void tower16_kernel(")
s = "#define AZ_KLOOP_PF 1\n" + s
open("az_tower16.hip", "w").write(s)
e = open("az_engine.hip").read()
old = "    } layouts[2] = {{tower16_tile_rows(HW), true}, {tower16_tile_rows(HW), false}};"
assert e.count(old) == 1
e = e.replace(old, "    } layouts[2] = {{tower16_tile_rows(HW), HW != 42}, {tower16_tile_rows(HW), false}};")
old = "        if (tower16_lds_bytes(HW, L.tr, prefix[i], L.db) <= kTowerLdsMax) {"
assert e.count(old) == 1
e = e.replace(old, "        if (tower16_lds_bytes(HW, L.tr, prefix[i], L.db) <= (HW == 42 ? 80 * 1024 : kTowerLdsMax)) {")
open("az_engine.hip", "w").write(e)
