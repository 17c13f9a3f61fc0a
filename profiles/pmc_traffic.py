#!/usr/bin/env python3
"""Fold pmc_traffic.sh's FETCH_SIZE / WRITE_SIZE passes into bytes per board.
Corrections per MI355X_MICROARCH.md (HBM/rocprofv3): counters in KiB; on
gfx950 FETCH_SIZE reports half the bytes of 16 B/lane streams -> x2."""
import csv
import glob
import json
import sys

out, B = sys.argv[1], int(sys.argv[2])
only = int(sys.argv[sys.argv.index("--only") + 1]) if "--only" in sys.argv else None


def per_kernel(d, name):
    acc = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if r["Counter_Name"] != name or "conv" not in k or "stem" in k:
                continue
            k = k.split("(")[0].replace("void ", "")
            acc.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, az_forward at B={B} boards",
       "correction": "fetch bytes = 2 x FETCH_SIZE KiB (gfx950, 16 B/lane streams); write = WRITE_SIZE KiB"}
for algo, key in ((0, "f16x2"), (1, "direct")):
    if only is not None and algo != only:
        continue
    f = per_kernel(f"{out}/fetch_{algo}", "FETCH_SIZE")
    w = per_kernel(f"{out}/write_{algo}", "WRITE_SIZE")
    per = {k: (2 * f[k] + w.get(k, 0.0)) * 1024 / B for k in f}
    res[key] = {"hbm_bytes_per_board": per,
                "mean_hbm_bytes_per_board_per_launch": sum(per.values()) / max(len(per), 1)}
print(json.dumps(res, indent=1))
