#!/usr/bin/env python3
"""Summarise rocprofv3 PMC databases (*.db): per kernel and counter, the mean
over dispatches (sum over the device's instances per dispatch).
Usage: python profiles/pmc_db.py <dir-or-db>... [--kernel SUBSTR] [--json]"""
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def load(paths):
    out = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for f in (sorted(glob.glob(os.path.join(p, "**", "*.db"), recursive=True)) if os.path.isdir(p) else [p]):
            c = sqlite3.connect(f)
            q = ("select dispatch_id, kernel_name, counter_name, sum(value), max(duration) from counters_collection "
                 "group by dispatch_id, kernel_name, counter_name")
            for _, k, name, v, dur in c.execute(q):
                out[k][name].append(v)
                out[k]["duration_ns"].append(dur)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ksub = None
    if "--kernel" in sys.argv:
        ksub = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != ksub]
    data = load(args)
    res = {}
    for k, cs in data.items():
        if ksub and ksub not in k:
            continue
        res[k] = {n: sum(v) / len(v) for n, v in cs.items()}
        res[k]["dispatches"] = len(cs.get("duration_ns", []))
    if "--json" in sys.argv:
        print(json.dumps(res, indent=1))
        return
    for k, cs in res.items():
        print(k[:110])
        for n in sorted(cs):
            print(f"   {n:28s} {cs[n]:.4g}")


if __name__ == "__main__":
    main()
