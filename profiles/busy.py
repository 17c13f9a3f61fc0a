#!/usr/bin/env python3
"""GPU busy fraction from a rocprofv3 kernel trace: union of kernel intervals
over the trace's last `window` seconds (steady state), per-kernel share, and
mean gap between consecutive kernels.  Usage: busy.py <kernel_trace.csv> [window_s]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:])
            for r in rows)
t_end = max(e for _, e, _ in iv)
t0 = t_end - int(win * 1e9)
iv = [(max(s, t0), e, n) for s, e, n in iv if e > t0]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t_end - iv[0][0]
print(f"window {span / 1e6:.1f} ms: GPU busy (union of kernels) {busy / span:.1%}")
tot = defaultdict(int)
cnt = defaultdict(int)
for s, e, n in iv:
    tot[n] += e - s
    cnt[n] += 1
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:12]:
    print(f"  {n:42s} {cnt[n]:7d} calls  {t / 1e6:8.1f} ms  avg {t / cnt[n] / 1e3:7.1f} us  ({t / span:.1%} of window)")
