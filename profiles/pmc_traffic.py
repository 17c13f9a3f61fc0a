#!/usr/bin/env python3
"""Fold pmc_traffic.sh's FETCH_SIZE / WRITE_SIZE passes into bytes per board
per launch of the forward's dominant kernel(s).
Corrections per MI355X_MICROARCH.md (HBM/rocprofv3): counters in KiB; on
gfx950 FETCH_SIZE reports half the bytes of 16 B/lane streams -> x2."""
import csv
import glob
import json
import sys

out, B = sys.argv[1], int(sys.argv[2])
only = int(sys.argv[sys.argv.index("--only") + 1]) if "--only" in sys.argv else None


def per_kernel(d, name, pat):
    acc = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if r["Counter_Name"] != name or pat not in k or "stem" in k:
                continue
            k = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            acc.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, az_forward at B={B} boards",
       "correction": "fetch bytes = 2 x FETCH_SIZE KiB (gfx950, 16 B/lane streams); write = WRITE_SIZE KiB"}
keys = {0: ("tower16", "tower16_kernel"), 1: ("direct", "conv3x3_mfma"), 2: ("f16x2", "conv16_kernel")}
if "--chess" in sys.argv:  # the chess network runs the per-layer fp16x2 convs under AZ_CONV_F16X2
    keys = {0: ("f16x2", "conv16_kernel"), 1: ("direct", "conv3x3_mfma")}
for algo, (key, pat) in keys.items():
    if only is not None and algo != only:
        continue
    import os
    if not os.path.isdir(f"{out}/fetch_{algo}"):
        continue
    f = per_kernel(f"{out}/fetch_{algo}", "FETCH_SIZE", pat)
    w = per_kernel(f"{out}/write_{algo}", "WRITE_SIZE", pat)
    per = {k: (2 * f[k] + w.get(k, 0.0)) * 1024 / B for k in f}
    res[key] = {"hbm_bytes_per_board": per,
                "mean_hbm_bytes_per_board_per_launch": sum(per.values()) / max(len(per), 1)}
print(json.dumps(res, indent=1))
