#!/usr/bin/env python3
"""Per-stream kernel chains from a rocprofv3 kernel trace: over the trace's
last `window` seconds, for each stream (Stream_Id, else Queue_Id) the summed
kernel time, the summed gaps between one kernel's end and the next kernel's
start on that stream, and the gap distribution -- how much of a lane's
simulation chain is launch/dependency latency rather than kernel time.
Usage: chain.py <kernel_trace.csv> [window_s] [skip_s] (the window ends skip_s before the trace's end)"""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
skip = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
key = "Stream_Id" if rows and "Stream_Id" in rows[0] else "Queue_Id"
t_end = max(int(r["End_Timestamp"]) for r in rows) - int(skip * 1e9)
t0 = t_end - int(win * 1e9)
by = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e > t0 and s < t_end:
        by[r[key]].append((s, e, r["Kernel_Name"].split("(")[0][-34:]))
print(f"streams by {key}, {win * 1e3:.0f} ms ending {skip * 1e3:.0f} ms before the trace's end")
for q, iv in sorted(by.items(), key=lambda x: -len(x[1])):
    iv.sort()
    busy = sum(e - s for s, e, _ in iv)
    gaps = [max(0, iv[i + 1][0] - iv[i][1]) for i in range(len(iv) - 1)]
    span = iv[-1][1] - iv[0][0]
    if len(iv) < 10:
        continue
    print(f"  {key} {q}: {len(iv)} kernels, span {span / 1e6:.1f} ms, kernel time {busy / span:.1%}, "
          f"gaps {sum(gaps) / span:.1%} (median {statistics.median(gaps) / 1e3:.1f} us, "
          f"p90 {sorted(gaps)[int(0.9 * len(gaps))] / 1e3:.1f} us)")
    after = defaultdict(list)
    for i in range(len(iv) - 1):
        after[iv[i + 1][2]].append(max(0, iv[i + 1][0] - iv[i][1]))
    for n, g in sorted(after.items(), key=lambda x: -sum(x[1]))[:8]:
        print(f"      gap before {n:34s} mean {sum(g) / len(g) / 1e3:6.1f} us  "
              f"median {statistics.median(g) / 1e3:6.1f} us  x{len(g)}")
    dur = defaultdict(list)
    for s, e, n in iv:
        dur[n].append(e - s)
    print("      kernel durations: " + "; ".join(
        f"{n.strip()} {sum(d) / len(d) / 1e3:.1f} us x{len(d)}"
        for n, d in sorted(dur.items(), key=lambda x: -sum(x[1]))[:9]))
