#!/usr/bin/env python3
"""Per-stream (lane) timeline from a rocprofv3 kernel trace: for the last
`window` seconds, each stream's busy fraction, time by kernel class, and the
mean gap between its consecutive kernels (launch/dependency bubbles).
Usage: lanes_timeline.py <kernel_trace.csv> [window_s]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
t_end = max(int(r["End_Timestamp"]) for r in rows)
t0 = t_end - int(win * 1e9)
streams = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e < t0:
        continue
    n = r["Kernel_Name"]
    k = "conv" if "conv_kernel" in n and "stem" not in n else n.split("(")[0].split("::")[-1].split("<")[0]
    streams[(r["Queue_Id"], r["Stream_Id"])].append((max(s, t0), e, k))
for sid, ev in sorted(streams.items()):
    ev.sort()
    busy = sum(e - s for s, e, _ in ev)
    gaps = [ev[i + 1][0] - ev[i][1] for i in range(len(ev) - 1)]
    by = defaultdict(int)
    for s, e, k in ev:
        by[k] += e - s
    span = t_end - t0
    print(f"queue {sid[0]} stream {sid[1]}: {len(ev)} kernels, busy {busy / span:.1%}, "
          f"mean gap {sum(gaps) / max(len(gaps), 1) / 1e3:.1f} us")
    for k, v in sorted(by.items(), key=lambda x: -x[1])[:8]:
        print(f"    {k:28s} {v / span:6.1%}")
