#!/usr/bin/env python3
"""Summarise a rocprofv3 collection (kernel trace/stats + FETCH_SIZE/WRITE_SIZE
passes) into the table committed under profiles/.

HBM bytes follow MI355X_MICROARCH.md's HBM/rocprofv3 section: counters are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced read, so fetched bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact
for 16 B/lane stores.  Usage: summarize.py <prof_dir> [boards_per_launch]
"""
import csv
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "")
    return name.split("(")[0][:60]


def stats(path):
    rows = list(csv.DictReader(open(path)))
    return [(short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
             float(r["Percentage"])) for r in rows]


def counters(path, name):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d = sys.argv[1]
    boards = float(sys.argv[2]) if len(sys.argv) > 2 else None
    st = stats(os.path.join(d, "trace", "run_kernel_stats.csv"))
    print("## Kernel time (rocprofv3 --kernel-trace --stats)\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for n, c, tot, avg, pct in st[:14]:
        print(f"| `{n}` | {c} | {tot / 1e6:.1f} | {avg / 1e3:.1f} | {pct:.2f} |")
    conv = [(c, tot) for n, c, tot, _, _ in st if "conv3x3_mfma" in n]
    if conv:
        calls = sum(c for c, _ in conv)
        tot = sum(t for _, t in conv)
        print(f"\nconv3x3_mfma (both variants): {calls} launches, average {tot / calls / 1e3:.1f} us")
    fetch_p = os.path.join(d, "fetch", "run_counter_collection.csv")
    write_p = os.path.join(d, "write", "run_counter_collection.csv")
    if os.path.exists(fetch_p) and os.path.exists(write_p):
        f, w = counters(fetch_p, "FETCH_SIZE"), counters(write_p, "WRITE_SIZE")
        print("\n## HBM traffic per launch (PMC, separate passes; fetch x2 gfx950 correction)\n")
        print("| kernel | FETCH_SIZE KiB | WRITE_SIZE KiB | HBM MB/launch (corrected) |"
              + (" KB/board |" if boards else ""))
        print("|---|---:|---:|---:|" + ("---:|" if boards else ""))
        for k in sorted(f, key=lambda k: -f[k]):
            if k not in w:
                continue
            mb = (2 * f[k] + w[k]) * 1024 / 1e6
            line = f"| `{k}` | {f[k]:.0f} | {w[k]:.0f} | {mb:.2f} |"
            if boards:
                line += f" {mb * 1e3 / boards:.2f} |"
            print(line)


if __name__ == "__main__":
    main()
